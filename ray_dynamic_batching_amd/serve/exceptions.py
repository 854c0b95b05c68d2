"""Serve-compatible exception types (reference: python/ray/serve/exceptions.py)."""


class RayServeException(Exception):
    pass


class BackPressureError(RayServeException):
    """Raised when a deployment already has max_queued_requests requests queued
    (reference router.py:116-131; HTTP 503 at the proxy)."""

    def __init__(self, num_queued_requests: int = 0, max_queued_requests: int = 0):
        self.num_queued_requests = num_queued_requests
        self.max_queued_requests = max_queued_requests
        super().__init__(f"Request dropped due to backpressure (num_queued_requests={num_queued_requests}, "
                         f"max_queued_requests={max_queued_requests}).")


class RequestCancelledError(RayServeException):
    pass


class DeploymentUnavailableError(RayServeException):
    pass


class ReplicaDiedError(RayServeException):
    pass


class RequestDroppedError(RayServeException):
    """The request's deadline (SLO) could not be met and it was dropped before
    execution (the fork's stale-request dropping, scheduler.py:281-283)."""

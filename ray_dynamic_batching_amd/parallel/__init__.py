"""Multi-GPU: collective-communication API (RCCL over xGMI via torch.distributed)
and tensor-parallel layers for TP replicas (Llama-3-8B TP=8)."""
from . import collective  # noqa: F401

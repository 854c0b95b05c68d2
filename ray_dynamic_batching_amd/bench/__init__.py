"""Benchmarks, workload generators and result logging."""

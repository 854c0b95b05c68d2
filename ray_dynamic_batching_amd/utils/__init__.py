"""Utilities: native-extension loading, config registry, logging, tracing, metrics."""

"""Triton model configuration messages (``inference.ModelConfig`` & co).

Runtime-built equivalent of the protoc output the reference copies in at wheel
build time (reference src/python/library/build_wheel.py:126-153).
"""
from ._descriptors import populate as _populate

_populate(globals(), "model_config.proto")

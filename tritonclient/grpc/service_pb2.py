"""KServe-v2 ``inference.GRPCInferenceService`` messages.

Runtime-built equivalent of ``grpc_service_pb2`` (reference
src/python/library/build_wheel.py:126-153).
"""
from . import model_config_pb2 as _model_config_pb2  # noqa: F401  (dependency)
from ._descriptors import populate as _populate

_populate(globals(), "grpc_service.proto")

"""Deprecated alias of ``tritonclient.grpc.service_pb2`` (reference package ``tritongrpcclient.grpc_service_pb2``)."""
import warnings

warnings.warn(
    "The package `tritongrpcclient.grpc_service_pb2` is deprecated and will be removed in a future version. Please use instead `tritonclient.grpc.service_pb2`",
    DeprecationWarning,
    stacklevel=2,
)

from tritonclient.grpc.service_pb2 import *  # noqa: E402,F401,F403

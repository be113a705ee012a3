"""Deprecated alias of ``tritonclient.grpc.service_pb2_grpc`` (reference package ``tritongrpcclient.grpc_service_pb2_grpc``)."""
import warnings

warnings.warn(
    "The package `tritongrpcclient.grpc_service_pb2_grpc` is deprecated and will be removed in a future version. Please use instead `tritonclient.grpc.service_pb2_grpc`",
    DeprecationWarning,
    stacklevel=2,
)

from tritonclient.grpc.service_pb2_grpc import *  # noqa: E402,F401,F403

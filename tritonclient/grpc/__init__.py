"""KServe-v2 gRPC client (reference tritonclient/grpc/__init__.py)."""
try:
    import grpc
except ModuleNotFoundError as error:  # pragma: no cover
    raise RuntimeError(
        "The installation does not include grpc support. Install grpcio."
    ) from error

from tritonclient.grpc import model_config_pb2, service_pb2, service_pb2_grpc  # noqa: F401
from tritonclient.utils import *  # noqa: F401,F403

from .._plugin import InferenceServerClientPlugin
from .._request import Request
from ._client import MAX_GRPC_MESSAGE_SIZE, CallContext, InferenceServerClient, KeepAliveOptions  # noqa: F401
from ._infer_input import InferInput
from ._infer_result import InferResult
from ._requested_output import InferRequestedOutput
from ._utils import raise_error, raise_error_grpc  # noqa: F401

# grpcio 1.43.0 .. 1.51.0 leak memory (reference grpc/__init__.py:53-64)
try:
    from packaging import version as _v

    if _v.parse("1.43.0") <= _v.parse(grpc.__version__) < _v.parse("1.51.1"):
        import warnings

        warnings.warn(
            f"Imported version of grpc is {grpc.__version__}. There is a memory "
            "leak in certain Python GRPC versions (1.43.0 to be specific). Please "
            "use versions <1.43.0 or >=1.51.1 to avoid leaks "
            "(see https://github.com/grpc/grpc/issues/28513)."
        )
except ImportError:  # pragma: no cover
    pass

__all__ = [
    "InferenceServerClientPlugin",
    "Request",
    "InferenceServerClient",
    "InferInput",
    "InferRequestedOutput",
    "InferResult",
    "KeepAliveOptions",
    "InferenceServerException",
]

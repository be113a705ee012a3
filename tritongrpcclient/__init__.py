"""Deprecated alias of ``tritonclient.grpc`` (reference package ``tritongrpcclient``)."""
import warnings

warnings.warn(
    "The package `tritongrpcclient` is deprecated and will be removed in a future version. Please use instead `tritonclient.grpc`",
    DeprecationWarning,
    stacklevel=2,
)

from tritonclient.grpc import *  # noqa: E402,F401,F403
from tritonclient.grpc import InferenceServerClient, InferInput, InferRequestedOutput, InferResult  # noqa: E402,F401

"""KServe-v2 REST client (reference tritonclient/http/__init__.py)."""
from tritonclient.utils import *  # noqa: F401,F403

from .._plugin import InferenceServerClientPlugin
from .._request import Request
from ._client import InferAsyncRequest, InferenceServerClient
from ._infer_input import InferInput
from ._infer_result import InferResult
from ._requested_output import InferRequestedOutput
from ._utils import InferenceServerException  # noqa: F401

__all__ = [
    "InferenceServerClientPlugin",
    "Request",
    "InferenceServerClient",
    "InferInput",
    "InferRequestedOutput",
    "InferResult",
    "InferAsyncRequest",
    "InferenceServerException",
]

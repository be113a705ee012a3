"""Deprecated alias of ``tritonclient.http`` (reference package ``tritonhttpclient``)."""
import warnings

warnings.warn(
    "The package `tritonhttpclient` is deprecated and will be removed in a future version. Please use instead `tritonclient.http`",
    DeprecationWarning,
    stacklevel=2,
)

from tritonclient.http import *  # noqa: E402,F401,F403
from tritonclient.http import InferenceServerClient, InferInput, InferRequestedOutput, InferResult  # noqa: E402,F401

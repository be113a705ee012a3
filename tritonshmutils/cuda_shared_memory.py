"""Deprecated alias of ``tritonclient.utils.cuda_shared_memory`` (reference package ``tritonshmutils.cuda_shared_memory``)."""
import warnings

warnings.warn(
    "The package `tritonshmutils.cuda_shared_memory` is deprecated and will be removed in a future version. Please use instead `tritonclient.utils.cuda_shared_memory`",
    DeprecationWarning,
    stacklevel=2,
)

from tritonclient.utils.cuda_shared_memory import *  # noqa: E402,F401,F403

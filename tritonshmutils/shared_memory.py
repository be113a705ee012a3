"""Deprecated alias of ``tritonclient.utils.shared_memory`` (reference package ``tritonshmutils.shared_memory``)."""
import warnings

warnings.warn(
    "The package `tritonshmutils.shared_memory` is deprecated and will be removed in a future version. Please use instead `tritonclient.utils.shared_memory`",
    DeprecationWarning,
    stacklevel=2,
)

from tritonclient.utils.shared_memory import *  # noqa: E402,F401,F403

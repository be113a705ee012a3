"""Deprecated alias of ``tritonclient.utils`` (reference package ``tritonclientutils``)."""
import warnings

warnings.warn(
    "The package `tritonclientutils` is deprecated and will be removed in a future version. Please use instead `tritonclient.utils`",
    DeprecationWarning,
    stacklevel=2,
)

from tritonclient.utils import *  # noqa: E402,F401,F403

"""Deprecated package (reference ``tritonshmutils``): use
``tritonclient.utils.shared_memory`` / ``tritonclient.utils.hip_shared_memory``."""
import warnings

warnings.warn(
    "The package `tritonshmutils` is deprecated and will be removed in a future version. Please use instead "
    "`tritonclient.utils.shared_memory` or `tritonclient.utils.cuda_shared_memory`",
    DeprecationWarning,
    stacklevel=2,
)

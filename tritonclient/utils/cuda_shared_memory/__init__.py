"""``tritonclient.utils.cuda_shared_memory`` — import-compatible alias.

On MI355X the device shared-memory implementation is HIP
(:mod:`tritonclient.utils.hip_shared_memory`); this module keeps the
reference's import path (reference tritonclient/utils/cuda_shared_memory) so
existing client code runs unchanged.
"""
from ..hip_shared_memory import *  # noqa: F401,F403
from ..hip_shared_memory import (  # noqa: F401
    CudaSharedMemoryException,
    HipSharedMemoryRegion as CudaSharedMemoryRegion,
    allocated_shared_memory_regions,
    as_shared_memory_tensor,
    create_shared_memory_region,
    destroy_shared_memory_region,
    get_contents_as_numpy,
    get_raw_handle,
    set_shared_memory_region,
    set_shared_memory_region_from_dlpack,
)

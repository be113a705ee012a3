"""Native compute path: HIP runtime glue + CDNA4 kernels (libtcamd_hip.so).

Everything here is a thin ctypes layer over in-tree shared objects built by
the top-level Makefile (``python __graft_entry__.py build``).  There is no
silent Python fallback on a GPU box: if ``libtcamd_hip.so`` is missing the
import of :mod:`triton_client_amd.ops.hip` raises.
"""

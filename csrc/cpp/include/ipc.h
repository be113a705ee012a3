// Device IPC handle type (reference src/c++/library/ipc.h:28-32).
// On MI355X the handle is a hipIpcMemHandle_t (64 bytes, the same size as
// cudaIpcMemHandle_t); it is typedef'd to the reference name for source
// compatibility of RegisterCudaSharedMemory() callers.  Builds without HIP get
// a 64-byte POD with the same layout.
#pragma once

#if defined(TRITON_ENABLE_GPU)
#include <hip/hip_runtime_api.h>
typedef hipIpcMemHandle_t cudaIpcMemHandle_t;
#else
struct cudaIpcMemHandle_t {
  char reserved[64];
};
#endif

// POSIX shared-memory helpers (reference src/c++/library/shm_utils.h:38-64).
#pragma once

#include <cstddef>
#include <string>

#include "common.h"

namespace triton { namespace client {

/// shm_open(O_CREAT) + ftruncate; returns the descriptor in *shm_fd.
Error CreateSharedMemoryRegion(std::string shm_key, size_t byte_size, int* shm_fd);
/// mmap [offset, offset+byte_size) of an open region.
Error MapSharedMemory(int shm_fd, size_t offset, size_t byte_size, void** shm_addr);
Error CloseSharedMemory(int shm_fd);
Error UnlinkSharedMemoryRegion(std::string shm_key);
Error UnmapSharedMemory(void* shm_addr, size_t byte_size);

}}  // namespace triton::client

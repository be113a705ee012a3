// POSIX shared-memory helpers (see include/shm_utils.h).
#include "shm_utils.h"

#include <errno.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>

namespace triton { namespace client {

Error
CreateSharedMemoryRegion(std::string shm_key, size_t byte_size, int* shm_fd)
{
  *shm_fd = shm_open(shm_key.c_str(), O_RDWR | O_CREAT, S_IRUSR | S_IWUSR);
  if (*shm_fd == -1) {
    return Error("unable to get shared memory descriptor for shared-memory key '" + shm_key + "': " +
                 std::strerror(errno));
  }
  if (ftruncate(*shm_fd, static_cast<off_t>(byte_size)) == -1) {
    return Error("unable to initialize shared-memory key '" + shm_key + "' to requested size " +
                 std::to_string(byte_size) + " bytes: " + std::strerror(errno));
  }
  return Error::Success;
}

Error
MapSharedMemory(int shm_fd, size_t offset, size_t byte_size, void** shm_addr)
{
  *shm_addr = mmap(nullptr, byte_size, PROT_READ | PROT_WRITE, MAP_SHARED, shm_fd, static_cast<off_t>(offset));
  if (*shm_addr == MAP_FAILED) {
    return Error("unable to process address space or shared-memory descriptor: " + std::to_string(shm_fd) + ": " +
                 std::strerror(errno));
  }
  return Error::Success;
}

Error
CloseSharedMemory(int shm_fd)
{
  if (close(shm_fd) == -1) {
    return Error("unable to close shared-memory descriptor: " + std::to_string(shm_fd));
  }
  return Error::Success;
}

Error
UnlinkSharedMemoryRegion(std::string shm_key)
{
  if (shm_unlink(shm_key.c_str()) == -1) {
    return Error("unable to unlink shared memory for key '" + shm_key + "': " + std::strerror(errno));
  }
  return Error::Success;
}

Error
UnmapSharedMemory(void* shm_addr, size_t byte_size)
{
  if (munmap(shm_addr, byte_size) == -1) {
    return Error("unable to munmap shared memory region: " + std::string(std::strerror(errno)));
  }
  return Error::Success;
}

}}  // namespace triton::client

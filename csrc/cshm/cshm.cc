// libcshm: POSIX system shared-memory regions behind a C ABI for ctypes.
//
// Capability parity with reference
// src/python/library/tritonclient/utils/shared_memory/shared_memory.{h,cc}
// (SharedMemoryRegionCreate/Set/GetSharedMemoryHandleInfo/Destroy, error codes
// -2..-6).  Design differences:
//   * the handle keeps the fd open only while mapping, and records the exact
//     mapping length so Destroy munmaps what was mapped;
//   * Set() bounds-checks offset+byte_size against the region (the reference
//     memcpy()s unchecked) and returns -7 on overflow;
//   * regions are mapped MAP_SHARED|MAP_POPULATE so the first inference does not
//     pay page faults inside the timed path.

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdint>
#include <cstring>
#include <string>

namespace {

struct ShmRegion {
  std::string triton_name;
  std::string key;
  void* base = nullptr;
  uint64_t byte_size = 0;
  uint64_t offset = 0;  // always 0 for regions this library creates
  int fd = -1;          // -1 once closed
};

}  // namespace

extern "C" {

// Error codes (shared with the Python binding's SharedMemoryException map)
//  0 ok, -2 shm_open, -3 ftruncate, -4 mmap, -5 shm_unlink, -6 munmap,
//  -7 out-of-range Set, -8 bad handle
int SharedMemoryRegionCreate(const char* triton_shm_name, const char* shm_key,
                             uint64_t byte_size, void** shm_handle) {
  if (shm_handle == nullptr || shm_key == nullptr) return -8;
  int fd = shm_open(shm_key, O_RDWR | O_CREAT, S_IRUSR | S_IWUSR);
  if (fd == -1) return -2;
  if (ftruncate(fd, static_cast<off_t>(byte_size)) == -1) {
    close(fd);
    return -3;
  }
  void* base = nullptr;
  if (byte_size > 0) {
    base = mmap(nullptr, byte_size, PROT_READ | PROT_WRITE,
                MAP_SHARED | MAP_POPULATE, fd, 0);
    if (base == MAP_FAILED) {
      close(fd);
      return -4;
    }
  }
  // The mapping keeps the object alive; the descriptor is no longer needed.
  close(fd);
  auto* r = new ShmRegion();
  r->triton_name = triton_shm_name ? triton_shm_name : "";
  r->key = shm_key;
  r->base = base;
  r->byte_size = byte_size;
  r->fd = -1;
  *shm_handle = r;
  return 0;
}

int SharedMemoryRegionSet(void* shm_handle, uint64_t offset, uint64_t byte_size,
                          const void* data) {
  auto* r = static_cast<ShmRegion*>(shm_handle);
  if (r == nullptr) return -8;
  if (offset > r->byte_size || byte_size > r->byte_size - offset) return -7;
  if (byte_size) std::memcpy(static_cast<char*>(r->base) + offset, data, byte_size);
  return 0;
}

int GetSharedMemoryHandleInfo(void* shm_handle, char** shm_addr,
                              const char** shm_key, int* shm_fd,
                              uint64_t* offset, uint64_t* byte_size) {
  auto* r = static_cast<ShmRegion*>(shm_handle);
  if (r == nullptr) return -8;
  if (shm_addr) *shm_addr = static_cast<char*>(r->base);
  if (shm_key) *shm_key = r->key.c_str();
  if (shm_fd) *shm_fd = r->fd;
  if (offset) *offset = r->offset;
  if (byte_size) *byte_size = r->byte_size;
  return 0;
}

int SharedMemoryRegionDestroy(void* shm_handle) {
  auto* r = static_cast<ShmRegion*>(shm_handle);
  if (r == nullptr) return -8;
  int rc = 0;
  if (r->base != nullptr && munmap(r->base, r->byte_size) == -1) rc = -6;
  if (shm_unlink(r->key.c_str()) == -1 && rc == 0) rc = -5;
  delete r;
  return rc;
}

// Map an EXISTING region (server side of the protocol): key/offset/byte_size
// as sent in a register request.  Returns -2/-4 on failure.
int SharedMemoryRegionOpen(const char* shm_key, uint64_t offset,
                           uint64_t byte_size, void** shm_handle) {
  if (shm_handle == nullptr || shm_key == nullptr) return -8;
  int fd = shm_open(shm_key, O_RDWR, S_IRUSR | S_IWUSR);
  if (fd == -1) return -2;
  struct stat st;
  if (fstat(fd, &st) == -1 ||
      static_cast<uint64_t>(st.st_size) < offset + byte_size) {
    close(fd);
    return -3;
  }
  uint64_t map_len = offset + byte_size;
  void* base = nullptr;
  if (map_len > 0) {
    base = mmap(nullptr, map_len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (base == MAP_FAILED) {
      close(fd);
      return -4;
    }
  }
  close(fd);
  auto* r = new ShmRegion();
  r->key = shm_key;
  r->base = base;
  r->byte_size = map_len;
  r->offset = offset;
  *shm_handle = r;
  return 0;
}

// Unmap without unlinking (server side).
int SharedMemoryRegionClose(void* shm_handle) {
  auto* r = static_cast<ShmRegion*>(shm_handle);
  if (r == nullptr) return -8;
  int rc = 0;
  if (r->base != nullptr && munmap(r->base, r->byte_size) == -1) rc = -6;
  delete r;
  return rc;
}

}  // extern "C"

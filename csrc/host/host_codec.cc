// libtcamd_host — host-side BYTES tensor codecs behind a C ABI.
//
// The reference serialises/deserialises BYTES tensors with per-element
// Python loops (tritonclient/utils/__init__.py:193-276).  These two routines
// do the byte shuffling in C++ so that Python only builds the element list:
//   pack: (concatenated payload, u32 lengths[n]) -> <u32 len><bytes>...
//   scan: serialized buffer -> (u64 payload offsets[n], u32 lengths[n])

#include <cstdint>
#include <cstring>

extern "C" {

// out must hold total_payload + 4*n bytes.
int tcamd_host_pack_bytes(const uint8_t* payload, const uint32_t* lens, uint64_t n, uint8_t* out) {
  uint64_t in = 0, o = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint32_t L = lens[i];
    out[o + 0] = (uint8_t)L;
    out[o + 1] = (uint8_t)(L >> 8);
    out[o + 2] = (uint8_t)(L >> 16);
    out[o + 3] = (uint8_t)(L >> 24);
    std::memcpy(out + o + 4, payload + in, L);
    in += L;
    o += 4 + (uint64_t)L;
  }
  return 0;
}

// Count elements of a serialized buffer; returns -1 when malformed.
int64_t tcamd_host_count_bytes(const uint8_t* buf, uint64_t nbytes) {
  uint64_t p = 0;
  int64_t n = 0;
  while (p < nbytes) {
    if (p + 4 > nbytes) return -1;
    uint32_t L;
    std::memcpy(&L, buf + p, 4);
    if (p + 4 + (uint64_t)L > nbytes) return -1;
    p += 4 + (uint64_t)L;
    ++n;
  }
  return n;
}

// Fill offsets/lengths for up to cap elements; returns the count or -1.
int64_t tcamd_host_scan_bytes(const uint8_t* buf, uint64_t nbytes, uint64_t* offs, uint32_t* lens,
                              uint64_t cap) {
  uint64_t p = 0;
  uint64_t n = 0;
  while (p < nbytes && n < cap) {
    if (p + 4 > nbytes) return -1;
    uint32_t L;
    std::memcpy(&L, buf + p, 4);
    if (p + 4 + (uint64_t)L > nbytes) return -1;
    offs[n] = p + 4;
    lens[n] = L;
    p += 4 + (uint64_t)L;
    ++n;
  }
  return (int64_t)n;
}

// As tcamd_host_scan_bytes over a buffer that may end mid-element (a prefix
// of a region copied to the host in chunks): stops at the first element that
// does not fit, returns the complete elements (up to cap) and, in *consumed,
// the bytes they span.
int64_t tcamd_host_scan_bytes_prefix(const uint8_t* buf, uint64_t nbytes, uint64_t* offs, uint32_t* lens,
                                     uint64_t cap, uint64_t* consumed) {
  uint64_t p = 0;
  uint64_t n = 0;
  while (n < cap && p + 4 <= nbytes) {
    uint32_t L;
    std::memcpy(&L, buf + p, 4);
    if (p + 4 + (uint64_t)L > nbytes) break;
    offs[n] = p + 4;
    lens[n] = L;
    p += 4 + (uint64_t)L;
    ++n;
  }
  *consumed = p;
  return (int64_t)n;
}

}  // extern "C"

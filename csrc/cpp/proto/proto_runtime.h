// Wire-format runtime for the classes emitted by tools/gen_cpp_proto.py.
// Protocol-buffer binary encoding (varint / fixed32 / fixed64 / length-
// delimited), proto3 packed repeated scalars, unknown-field skipping and
// text-format printing helpers.  Header-only, no dependencies.
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <type_traits>

namespace tcamd_pb {

enum WireType : int { kVarint = 0, k64 = 1, kLen = 2, k32 = 5 };

struct Reader {
  const char* p;
};

inline void PutVarint(std::string* out, uint64_t v) {
  char buf[10];
  int n = 0;
  while (v >= 0x80) {
    buf[n++] = static_cast<char>((v & 0x7f) | 0x80);
    v >>= 7;
  }
  buf[n++] = static_cast<char>(v);
  out->append(buf, n);
}

inline void PutTag(std::string* out, uint32_t field, int wt) {
  PutVarint(out, (static_cast<uint64_t>(field) << 3) | static_cast<uint64_t>(wt));
}

inline void PutBytes(std::string* out, uint32_t field, const std::string& s) {
  PutTag(out, field, kLen);
  PutVarint(out, s.size());
  out->append(s);
}

template <typename M>
inline void EncodeMessage(std::string* out, uint32_t field, const M& m) {
  std::string sub;
  m.Encode(&sub);
  PutBytes(out, field, sub);
}

inline void PutFixed32Raw(std::string* out, uint32_t v) {
  char b[4];
  std::memcpy(b, &v, 4);  // little-endian host (x86-64 / CDNA hosts)
  out->append(b, 4);
}
inline void PutFixed64Raw(std::string* out, uint64_t v) {
  char b[8];
  std::memcpy(b, &v, 8);
  out->append(b, 8);
}

// ---- typed puts (with tag) ---------------------------------------------------
inline void PutVarintS64(std::string* o, uint32_t f, int64_t v) { PutTag(o, f, kVarint); PutVarint(o, static_cast<uint64_t>(v)); }
inline void PutVarintU64(std::string* o, uint32_t f, uint64_t v) { PutTag(o, f, kVarint); PutVarint(o, v); }
inline void PutVarintS32(std::string* o, uint32_t f, int32_t v) { PutTag(o, f, kVarint); PutVarint(o, static_cast<uint64_t>(static_cast<int64_t>(v))); }
inline void PutVarintU32(std::string* o, uint32_t f, uint32_t v) { PutTag(o, f, kVarint); PutVarint(o, v); }
inline void PutVarintBool(std::string* o, uint32_t f, bool v) { PutTag(o, f, kVarint); PutVarint(o, v ? 1 : 0); }
inline void PutZigZag32(std::string* o, uint32_t f, int32_t v) { PutTag(o, f, kVarint); PutVarint(o, (static_cast<uint32_t>(v) << 1) ^ static_cast<uint32_t>(v >> 31)); }
inline void PutZigZag64(std::string* o, uint32_t f, int64_t v) { PutTag(o, f, kVarint); PutVarint(o, (static_cast<uint64_t>(v) << 1) ^ static_cast<uint64_t>(v >> 63)); }
inline void PutFixed32U(std::string* o, uint32_t f, uint32_t v) { PutTag(o, f, k32); PutFixed32Raw(o, v); }
inline void PutFixed32S(std::string* o, uint32_t f, int32_t v) { PutTag(o, f, k32); PutFixed32Raw(o, static_cast<uint32_t>(v)); }
inline void PutFixed64U(std::string* o, uint32_t f, uint64_t v) { PutTag(o, f, k64); PutFixed64Raw(o, v); }
inline void PutFixed64S(std::string* o, uint32_t f, int64_t v) { PutTag(o, f, k64); PutFixed64Raw(o, static_cast<uint64_t>(v)); }
inline void PutFixed32Float(std::string* o, uint32_t f, float v) { uint32_t u; std::memcpy(&u, &v, 4); PutTag(o, f, k32); PutFixed32Raw(o, u); }
inline void PutFixed64Double(std::string* o, uint32_t f, double v) { uint64_t u; std::memcpy(&u, &v, 8); PutTag(o, f, k64); PutFixed64Raw(o, u); }

// ---- packed (no tag) ----------------------------------------------------------
inline void PutPackedVarintS64(std::string* o, int64_t v) { PutVarint(o, static_cast<uint64_t>(v)); }
inline void PutPackedVarintU64(std::string* o, uint64_t v) { PutVarint(o, v); }
inline void PutPackedVarintS32(std::string* o, int32_t v) { PutVarint(o, static_cast<uint64_t>(static_cast<int64_t>(v))); }
inline void PutPackedVarintU32(std::string* o, uint32_t v) { PutVarint(o, v); }
inline void PutPackedVarintBool(std::string* o, bool v) { PutVarint(o, v ? 1 : 0); }
inline void PutPackedZigZag32(std::string* o, int32_t v) { PutVarint(o, (static_cast<uint32_t>(v) << 1) ^ static_cast<uint32_t>(v >> 31)); }
inline void PutPackedZigZag64(std::string* o, int64_t v) { PutVarint(o, (static_cast<uint64_t>(v) << 1) ^ static_cast<uint64_t>(v >> 63)); }
inline void PutPackedFixed32U(std::string* o, uint32_t v) { PutFixed32Raw(o, v); }
inline void PutPackedFixed32S(std::string* o, int32_t v) { PutFixed32Raw(o, static_cast<uint32_t>(v)); }
inline void PutPackedFixed64U(std::string* o, uint64_t v) { PutFixed64Raw(o, v); }
inline void PutPackedFixed64S(std::string* o, int64_t v) { PutFixed64Raw(o, static_cast<uint64_t>(v)); }
inline void PutPackedFixed32Float(std::string* o, float v) { uint32_t u; std::memcpy(&u, &v, 4); PutFixed32Raw(o, u); }
inline void PutPackedFixed64Double(std::string* o, double v) { uint64_t u; std::memcpy(&u, &v, 8); PutFixed64Raw(o, u); }

// ---- decoding -----------------------------------------------------------------
inline bool GetVarint(Reader* r, const char* end, uint64_t* v) {
  uint64_t result = 0;
  for (int shift = 0; shift < 64; shift += 7) {
    if (r->p >= end) return false;
    uint8_t b = static_cast<uint8_t>(*r->p++);
    result |= static_cast<uint64_t>(b & 0x7f) << shift;
    if (!(b & 0x80)) {
      *v = result;
      return true;
    }
  }
  return false;
}

inline bool GetTag(Reader* r, const char* end, uint32_t* field, int* wt) {
  uint64_t t;
  if (!GetVarint(r, end, &t)) return false;
  *field = static_cast<uint32_t>(t >> 3);
  *wt = static_cast<int>(t & 7);
  return *field != 0;
}

inline bool GetLength(Reader* r, const char* end, int wt, const char** sub_end) {
  if (wt != kLen) return false;
  uint64_t n;
  if (!GetVarint(r, end, &n)) return false;
  if (n > static_cast<uint64_t>(end - r->p)) return false;
  *sub_end = r->p + n;
  return true;
}

inline bool GetBytes(Reader* r, const char* end, int wt, std::string* s) {
  const char* e;
  if (!GetLength(r, end, wt, &e)) return false;
  s->assign(r->p, e - r->p);
  r->p = e;
  return true;
}

inline bool GetFixed32Raw(Reader* r, const char* end, uint32_t* v) {
  if (end - r->p < 4) return false;
  std::memcpy(v, r->p, 4);
  r->p += 4;
  return true;
}
inline bool GetFixed64Raw(Reader* r, const char* end, uint64_t* v) {
  if (end - r->p < 8) return false;
  std::memcpy(v, r->p, 8);
  r->p += 8;
  return true;
}

inline bool SkipField(Reader* r, const char* end, int wt) {
  uint64_t v;
  switch (wt) {
    case kVarint: return GetVarint(r, end, &v);
    case k64: if (end - r->p < 8) return false; r->p += 8; return true;
    case k32: if (end - r->p < 4) return false; r->p += 4; return true;
    case kLen: { const char* e; if (!GetLength(r, end, wt, &e)) return false; r->p = e; return true; }
    default: return false;
  }
}

#define TCAMD_PB_VARINT_GET(NAME, T, CONV)                                                        \
  inline bool GetPacked##NAME(Reader* r, const char* end, T* out) {                            \
    uint64_t v; if (!GetVarint(r, end, &v)) return false; *out = CONV; return true;            \
  }                                                                                            \
  inline bool Get##NAME(Reader* r, const char* end, int wt, T* out) {                          \
    return wt == kVarint && GetPacked##NAME(r, end, out);                                    \
  }
TCAMD_PB_VARINT_GET(VarintS64, int64_t, static_cast<int64_t>(v))
TCAMD_PB_VARINT_GET(VarintU64, uint64_t, v)
TCAMD_PB_VARINT_GET(VarintS32, int32_t, static_cast<int32_t>(v))
TCAMD_PB_VARINT_GET(VarintU32, uint32_t, static_cast<uint32_t>(v))
TCAMD_PB_VARINT_GET(VarintBool, bool, v != 0)
TCAMD_PB_VARINT_GET(ZigZag32, int32_t, static_cast<int32_t>((static_cast<uint32_t>(v) >> 1) ^ (~(static_cast<uint32_t>(v) & 1) + 1)))
TCAMD_PB_VARINT_GET(ZigZag64, int64_t, static_cast<int64_t>((v >> 1) ^ (~(v & 1) + 1)))
#undef TCAMD_PB_VARINT_GET

#define TCAMD_PB_FIXED_GET(NAME, T, RAW, RAWT, W)                                                \
  inline bool GetPacked##NAME(Reader* r, const char* end, T* out) {                            \
    RAWT u; if (!RAW(r, end, &u)) return false; std::memcpy(out, &u, sizeof(T)); return true;  \
  }                                                                                            \
  inline bool Get##NAME(Reader* r, const char* end, int wt, T* out) {                          \
    return wt == W && GetPacked##NAME(r, end, out);                                          \
  }
TCAMD_PB_FIXED_GET(Fixed32U, uint32_t, GetFixed32Raw, uint32_t, k32)
TCAMD_PB_FIXED_GET(Fixed32S, int32_t, GetFixed32Raw, uint32_t, k32)
TCAMD_PB_FIXED_GET(Fixed32Float, float, GetFixed32Raw, uint32_t, k32)
TCAMD_PB_FIXED_GET(Fixed64U, uint64_t, GetFixed64Raw, uint64_t, k64)
TCAMD_PB_FIXED_GET(Fixed64S, int64_t, GetFixed64Raw, uint64_t, k64)
TCAMD_PB_FIXED_GET(Fixed64Double, double, GetFixed64Raw, uint64_t, k64)
#undef TCAMD_PB_FIXED_GET

// ---- text format ----------------------------------------------------------------
inline void PrintIndent(std::string* out, int indent) { out->append(static_cast<size_t>(indent) * 2, ' '); }

inline void AppendEscaped(std::string* out, const std::string& s) {
  for (unsigned char c : s) {
    switch (c) {
      case '\n': out->append("\\n"); break;
      case '\r': out->append("\\r"); break;
      case '\t': out->append("\\t"); break;
      case '"': out->append("\\\""); break;
      case '\\': out->append("\\\\"); break;
      default:
        if (c < 0x20 || c >= 0x7f) {
          char b[8];
          std::snprintf(b, sizeof(b), "\\%03o", c);
          out->append(b);
        } else {
          out->push_back(static_cast<char>(c));
        }
    }
  }
}

template <typename T>
inline void AppendNumber(std::string* out, T v) {
  if constexpr (std::is_floating_point<T>::value) {
    char b[64];
    std::snprintf(b, sizeof(b), "%.9g", static_cast<double>(v));
    out->append(b);
  } else {
    out->append(std::to_string(v));
  }
}

}  // namespace tcamd_pb

// Socket / TLS / HTTP-1.1 plumbing shared by the C++ HTTP client and perf tool.
#pragma once

#include <sys/uio.h>

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

typedef struct ssl_st SSL;
typedef struct ssl_ctx_st SSL_CTX;

namespace triton { namespace client {

struct TlsConfig {
  bool enabled = false;
  bool verify_peer = true;
  bool verify_host = true;
  std::string ca_info, cert, key;
  bool cert_der = false, key_der = false;
  std::string alpn;  // ALPN protocol to offer ("h2" for gRPC: servers refuse TLS without it)
};

/// A connected TCP (optionally TLS) stream socket.
class Socket {
 public:
  Socket() = default;
  ~Socket();
  Socket(const Socket&) = delete;
  Socket& operator=(const Socket&) = delete;

  /// Blocking connect with timeout (0 = none); returns "" or an error message.
  std::string Connect(const std::string& host, int port, uint64_t timeout_us, const TlsConfig& tls);
  void Close();
  bool IsOpen() const { return fd_ >= 0; }
  int fd() const { return fd_; }
  bool IsTls() const { return ssl_ != nullptr; }
  void SetNonBlocking(bool nb);

  /// writev semantics: returns bytes written, 0 on would-block, -1 on error.
  ssize_t Writev(struct iovec* iov, int iovcnt);
  /// returns bytes read, 0 on EOF, -1 on error, -2 on would-block.
  ssize_t Read(void* buf, size_t n);
  /// wait until readable/writable; returns false on timeout/error.
  bool Wait(bool for_write, int64_t timeout_us);

 private:
  int fd_ = -1;
  SSL* ssl_ = nullptr;
  SSL_CTX* ctx_ = nullptr;
};

/// Incremental HTTP/1.1 response parser (Content-Length and chunked bodies).
class HttpResponseParser {
 public:
  enum class State { Headers, Body, Chunked, Done, Error };
  void Reset(bool head_request = false);
  /// Feed bytes; returns bytes consumed. Check state() afterwards.
  size_t Feed(const char* data, size_t n);
  State state() const { return state_; }
  long status() const { return status_; }
  const std::map<std::string, std::string>& headers() const { return headers_; }
  std::string& body() { return body_; }
  bool keep_alive() const { return keep_alive_; }
  const std::string& error() const { return error_; }
  /// time the first body byte arrived (ns, steady) — RECV_START analogue
  uint64_t first_byte_ns() const { return first_byte_ns_; }

 private:
  bool ParseHeaders();
  State state_ = State::Headers;
  std::string head_;
  std::map<std::string, std::string> headers_;
  std::string body_;
  size_t content_length_ = 0;
  bool has_length_ = false;
  long status_ = 0;
  bool keep_alive_ = true;
  bool head_request_ = false;
  std::string error_;
  // chunked state
  size_t chunk_left_ = 0;
  int chunk_phase_ = 0;  // 0 size line, 1 data, 2 CRLF, 3 trailers
  std::string line_;
  uint64_t first_byte_ns_ = 0;
};

/// Lower-cased header lookup.
std::string HeaderValue(const std::map<std::string, std::string>& h, const std::string& name);

/// zlib helpers; gzip selects the gzip wrapper (windowBits 15|16).
bool Compress(const std::vector<std::pair<const char*, size_t>>& parts, bool gzip, std::string* out);
bool Decompress(const std::string& in, std::string* out);

std::string Base64Encode(const void* data, size_t n);
/// Base64 with the reference's libb64 framing (src/c++/library/cencode.c:
/// 78-81,106): a '\n' after every 72 output characters of full 3-byte groups,
/// then the padding, then a terminating '\n'.  The reference HTTP client sends
/// exactly these bytes in the LoadModel file-override values and the CUDA-shm
/// register "b64" handle, so ours does too (byte-compatible request bodies).
std::string Base64EncodeLibb64(const void* data, size_t n);
bool Base64Decode(const std::string& in, std::string* out);
std::string UrlEncode(const std::string& s);

}}  // namespace triton::client

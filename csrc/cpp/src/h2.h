// gRPC-over-HTTP/2 channel for the C++ gRPC client (no grpc++ on the box).
//
// One TCP (optionally TLS) connection per channel, an nghttp2 client session
// for framing/HPACK/flow control, and ONE I/O thread that owns the session:
// other threads hand it work through a queue + eventfd.  Calls are gRPC
// length-prefixed messages (1-byte compressed flag + 4-byte BE length) over
// an HTTP/2 stream; status comes from the grpc-status / grpc-message
// trailers.  Unary calls and bidirectional streams share the machinery.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "net.h"

namespace triton { namespace client {

enum class GrpcCompression { NONE = 0, DEFLATE = 1, GZIP = 2 };

struct GrpcStatus {
  int code = 0;  // 0 = OK; grpc::StatusCode numbering
  std::string message;
  bool ok() const { return code == 0; }
  std::string CodeName() const;
};

struct H2ChannelOptions {
  TlsConfig tls;
  int64_t keepalive_time_ms = INT32_MAX;
  int64_t keepalive_timeout_ms = 20000;
  bool keepalive_permit_without_calls = false;
  int http2_max_pings_without_data = 2;
  uint32_t initial_window = (1u << 31) - 1;
  size_t max_message_bytes = INT32_MAX;
};

/// Per-call callbacks, all invoked on the channel's I/O thread.
struct H2CallHandlers {
  std::function<void(std::string&& message)> on_message;
  std::function<void(const GrpcStatus& status)> on_close;
};

class H2Call;

class H2Channel : public std::enable_shared_from_this<H2Channel> {
 public:
  static std::shared_ptr<H2Channel> Create(const std::string& host, int port, const H2ChannelOptions& opts,
                                           std::string* err);
  ~H2Channel();

  /// Start a call on `path` (e.g. "/inference.GRPCInferenceService/ModelInfer").
  /// For unary calls pass the request and `half_close=true`.
  std::shared_ptr<H2Call> StartCall(
      const std::string& path, const std::vector<std::pair<std::string, std::string>>& metadata,
      uint64_t timeout_us, GrpcCompression compression, H2CallHandlers handlers);

  bool Healthy() const { return !dead_.load(); }
  const std::string& authority() const { return authority_; }

 private:
  friend class H2Call;
  H2Channel() = default;
  void Loop();
  void LoopBody();
  void Wake();
  void Post(std::function<void()> fn);
  void FailAll(const std::string& why);
  bool FlushSend();

  Socket sock_;
  std::string authority_;
  H2ChannelOptions opts_;
  void* session_ = nullptr;  // nghttp2_session*
  int evfd_ = -1;
  std::thread io_;
  std::mutex mu_;
  std::deque<std::function<void()>> tasks_;
  std::atomic<bool> stop_{false};
  std::atomic<bool> dead_{false};
  bool delete_on_exit_ = false;  // io thread only
  std::string dead_reason_;
  std::unordered_map<int32_t, std::shared_ptr<H2Call>> calls_;
  std::string sendbuf_;
  size_t sendpos_ = 0;
  uint64_t last_activity_ns_ = 0;
  uint64_t ping_sent_ns_ = 0;

  // nghttp2 callbacks need access
 public:
  void OnStreamClose(int32_t stream_id, uint32_t error_code);
  void OnHeader(int32_t stream_id, const std::string& name, const std::string& value);
  void OnData(int32_t stream_id, const uint8_t* data, size_t len);
  void OnFrameRecv(int32_t stream_id, bool end_stream, bool is_headers);
  void OnPingAck() { ping_sent_ns_ = 0; }
  long ReadBody(int32_t stream_id, uint8_t* buf, size_t length, uint32_t* data_flags);
};

/// One gRPC call (unary or streaming).  Thread-safe writers.
class H2Call : public std::enable_shared_from_this<H2Call> {
 public:
  /// Queue one request message (serialised protobuf).
  void Write(std::string&& message);
  /// A message already carrying its 5-byte gRPC prefix (uncompressed calls only).
  void WriteFramed(std::string&& framed);
  /// No more messages from the client (END_STREAM).
  void WritesDone();
  /// Abort the call (RST_STREAM CANCEL); on_close gets CANCELLED.
  void Cancel();

 private:
  friend class H2Channel;
  std::weak_ptr<H2Channel> chan_;
  int32_t stream_id_ = -1;
  H2CallHandlers handlers_;
  GrpcCompression compression_ = GrpcCompression::NONE;
  // send side (I/O thread only after start)
  std::deque<std::string> out_;
  size_t out_pos_ = 0;
  bool writes_done_ = false;
  bool deferred_ = false;
  // receive side
  std::string inbuf_;
  bool resp_compressed_gzip_ = false, resp_compressed_deflate_ = false;
  int http_status_ = 0;
  bool have_grpc_status_ = false;
  GrpcStatus status_;
  bool closed_ = false;
  uint64_t deadline_ns_ = 0;
  bool cancelled_ = false;
};

/// Encode one gRPC frame (optionally compressed).
bool GrpcFrame(const std::string& message, GrpcCompression comp, std::string* out);

}}  // namespace triton::client

// triton::client core types — MI355X-native C++ client library.
//
// Public API parity with reference src/c++/library/common.h:61-673
// (Error, InferStat, InferenceServerClient, InferOptions, InferInput,
// InferRequestedOutput, InferResult, RequestTimers, InferRequest).  The
// implementation is new: input buffers form a zero-copy scatter list that
// the HTTP transport hands to writev() directly, and timers use the steady
// monotonic clock (the reference uses high_resolution_clock).
#pragma once

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <limits>
#include <list>
#include <mutex>
#include <ostream>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>


/// Friend hook (reference src/c++/library/common.h:42-47,358-361,462-464): a
/// translation unit that defines TRITON_INFERENCE_SERVER_CLIENT_CLASS before
/// including this header (an in-process backend, a white-box test) is granted
/// access to the private state of the request/tensor classes.
#ifdef TRITON_INFERENCE_SERVER_CLIENT_CLASS
#define TC_CLIENT_FRIEND friend class TRITON_INFERENCE_SERVER_CLIENT_CLASS;
#else
#define TC_CLIENT_FRIEND
#endif

namespace triton { namespace client {

constexpr char kInferHeaderContentLengthHTTPHeader[] = "Inference-Header-Content-Length";
constexpr char kContentLengthHTTPHeader[] = "Content-Length";
constexpr int MAX_GRPC_MESSAGE_SIZE = INT32_MAX;

class InferResult;
class InferRequest;
class RequestTimers;

//==============================================================================
/// Error status: empty message == success.
class Error {
 public:
  explicit Error(const std::string& msg = "");
  const std::string& Message() const { return msg_; }
  bool IsOk() const { return msg_.empty(); }
  static const Error Success;

 private:
  friend std::ostream& operator<<(std::ostream&, const Error&);
  std::string msg_;
};

//==============================================================================
/// Cumulative client-side statistics of completed requests.
struct InferStat {
  size_t completed_request_count = 0;
  uint64_t cumulative_total_request_time_ns = 0;
  uint64_t cumulative_send_time_ns = 0;
  uint64_t cumulative_receive_time_ns = 0;
};

//==============================================================================
/// Base of the protocol clients (worker thread + stats).
class InferenceServerClient {
 public:
  using OnCompleteFn = std::function<void(InferResult*)>;
  using OnMultiCompleteFn = std::function<void(std::vector<InferResult*>)>;

  explicit InferenceServerClient(bool verbose) : verbose_(verbose), exiting_(false) {}
  virtual ~InferenceServerClient() = default;

  /// Snapshot of the cumulative statistics of this client.
  Error ClientInferStat(InferStat* infer_stat) const;

 protected:
  Error UpdateInferStat(const RequestTimers& timer);

  bool verbose_;
  std::thread worker_;
  mutable std::mutex mutex_;
  std::condition_variable cv_;
  bool exiting_;
  InferStat infer_stat_;
};

//==============================================================================
/// A typed custom request parameter ("string", "int", "bool", "double").
struct RequestParameter {
  std::string name;
  std::string value;
  std::string type;
};

//==============================================================================
/// Per-request options.
struct InferOptions {
  explicit InferOptions(const std::string& model_name)
      : model_name_(model_name), model_version_(""), request_id_(""), sequence_id_(0),
        sequence_id_str_(""), sequence_start_(false), sequence_end_(false), priority_(0),
        server_timeout_(0), client_timeout_(0), triton_enable_empty_final_response_(false)
  {
  }
  std::string model_name_;
  std::string model_version_;
  std::string request_id_;
  uint64_t sequence_id_;
  std::string sequence_id_str_;
  bool sequence_start_;
  bool sequence_end_;
  uint64_t priority_;
  uint64_t server_timeout_;  // microseconds, sent to the server
  uint64_t client_timeout_;  // microseconds, enforced by the client
  bool triton_enable_empty_final_response_;
  std::unordered_map<std::string, RequestParameter> request_parameters;
};

//==============================================================================
/// An input tensor: shape/datatype plus a zero-copy list of user buffers,
/// or a shared-memory reference.
class InferInput {
 public:
  static Error Create(
      InferInput** infer_input, const std::string& name, const std::vector<int64_t>& dims,
      const std::string& datatype);

  const std::string& Name() const { return name_; }
  const std::string& Datatype() const { return datatype_; }
  const std::vector<int64_t>& Shape() const { return shape_; }
  Error SetShape(const std::vector<int64_t>& dims);
  /// Drop all appended buffers / shared-memory settings.
  Error Reset();
  /// Append a buffer (NOT copied: must stay valid until the request completes).
  Error AppendRaw(const std::vector<uint8_t>& input);
  Error AppendRaw(const uint8_t* input, size_t input_byte_size);
  Error SetSharedMemory(const std::string& name, size_t byte_size, size_t offset = 0);
  bool IsSharedMemory() const { return io_type_ == SHARED_MEMORY; }
  Error SharedMemoryInfo(std::string* name, size_t* byte_size, size_t* offset) const;
  /// Serialise strings as BYTES elements (<u32 len><bytes>), owned by the input.
  Error AppendFromString(const std::vector<std::string>& input);
  /// Pointer to the data when it is a single contiguous buffer.
  Error RawData(const uint8_t** buf, size_t* byte_size);
  Error ByteSize(size_t* byte_size) const;
  bool BinaryData() const { return binary_data_; }
  Error SetBinaryData(const bool binary_data);

  // -- transport-facing (used by the HTTP/gRPC clients) ----------------------
  /// The appended buffers in order.
  const std::vector<const uint8_t*>& Buffers() const { return bufs_; }
  const std::vector<size_t>& BufferSizes() const { return buf_byte_sizes_; }
  Error PrepareForRequest();
  /// Copy up to `size` bytes into `buf` from the current cursor.
  Error GetNext(uint8_t* buf, size_t size, size_t* input_bytes, bool* end_of_input);
  /// Zero-copy cursor over the buffers.
  Error GetNext(const uint8_t** buf, size_t* input_bytes, bool* end_of_input);

 private:
  TC_CLIENT_FRIEND
  InferInput(const std::string& name, const std::vector<int64_t>& dims, const std::string& datatype);

  std::string name_;
  std::vector<int64_t> shape_;
  std::string datatype_;
  size_t byte_size_;
  size_t bufs_idx_, buf_pos_;
  std::vector<const uint8_t*> bufs_;
  std::vector<size_t> buf_byte_sizes_;
  std::list<std::string> str_bufs_;
  enum IOType { NONE, RAW, SHARED_MEMORY };
  IOType io_type_;
  std::string shm_name_;
  size_t shm_offset_;
  bool binary_data_{true};
};

//==============================================================================
class InferRequestedOutput {
 public:
  static Error Create(
      InferRequestedOutput** infer_output, const std::string& name, const size_t class_count = 0,
      const std::string& datatype = "");
  const std::string& Name() const { return name_; }
  const std::string& Datatype() const { return datatype_; }
  size_t ClassificationCount() const { return class_count_; }
  Error SetSharedMemory(const std::string& region_name, const size_t byte_size, const size_t offset = 0);
  Error UnsetSharedMemory();
  bool IsSharedMemory() const { return io_type_ == SHARED_MEMORY; }
  Error SharedMemoryInfo(std::string* name, size_t* byte_size, size_t* offset) const;
  bool BinaryData() const { return binary_data_; }
  Error SetBinaryData(const bool binary_data);

 private:
  TC_CLIENT_FRIEND
  explicit InferRequestedOutput(const std::string& name, const std::string& datatype, const size_t class_count = 0);
  std::string name_;
  std::string datatype_;
  size_t class_count_;
  enum IOType { NONE, RAW, SHARED_MEMORY };
  IOType io_type_;
  std::string shm_name_;
  size_t shm_byte_size_;
  size_t shm_offset_;
  bool binary_data_{true};
};

//==============================================================================
/// Result of one inference (protocol-specific subclasses).
class InferResult {
 public:
  virtual ~InferResult() = default;
  virtual Error ModelName(std::string* name) const = 0;
  virtual Error ModelVersion(std::string* version) const = 0;
  virtual Error Id(std::string* id) const = 0;
  virtual Error Shape(const std::string& output_name, std::vector<int64_t>* shape) const = 0;
  virtual Error Datatype(const std::string& output_name, std::string* datatype) const = 0;
  virtual Error RawData(const std::string& output_name, const uint8_t** buf, size_t* byte_size) const = 0;
  virtual Error IsFinalResponse(bool* is_final_response) const = 0;
  virtual Error IsNullResponse(bool* is_null_response) const = 0;
  virtual Error StringData(const std::string& output_name, std::vector<std::string>* string_result) const = 0;
  virtual std::string DebugString() const = 0;
  virtual Error RequestStatus() const = 0;
};

//==============================================================================
/// Six-point request timeline (ns, steady clock).
class RequestTimers {
 public:
  enum class Kind { REQUEST_START, REQUEST_END, SEND_START, SEND_END, RECV_START, RECV_END, COUNT__ };

  RequestTimers() { Reset(); }
  void Reset() { std::memset(timestamps_, 0, sizeof(timestamps_)); }
  uint64_t Timestamp(Kind kind) const { return timestamps_[static_cast<size_t>(kind)]; }
  uint64_t CaptureTimestamp(Kind kind)
  {
    uint64_t& ts = timestamps_[static_cast<size_t>(kind)];
    ts = Now();
    return ts;
  }
  void SetTimestamp(Kind kind, uint64_t ts) { timestamps_[static_cast<size_t>(kind)] = ts; }
  uint64_t Duration(Kind start, Kind end) const
  {
    const uint64_t s = timestamps_[static_cast<size_t>(start)];
    const uint64_t e = timestamps_[static_cast<size_t>(end)];
    if (s == 0 || e == 0 || s > e) return (std::numeric_limits<uint64_t>::max)();
    return e - s;
  }
  static uint64_t Now()
  {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }

 private:
  uint64_t timestamps_[static_cast<size_t>(Kind::COUNT__)];
};

//==============================================================================
class InferRequest {
 public:
  InferRequest(InferenceServerClient::OnCompleteFn callback = nullptr, const bool verbose = false)
      : callback_(callback), verbose_(verbose)
  {
  }
  virtual ~InferRequest() = default;
  RequestTimers& Timer() { return timer_; }

 protected:
  InferenceServerClient::OnCompleteFn callback_;
  const bool verbose_;

 private:
  RequestTimers timer_;
};

/// Element byte size of a fixed-size datatype; 0 for BYTES/unknown.
size_t DatatypeByteSize(const std::string& datatype);

}}  // namespace triton::client

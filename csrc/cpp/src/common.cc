// Implementation of the triton::client core types (see include/common.h).
#include "common.h"

namespace triton { namespace client {

const Error Error::Success("");

Error::Error(const std::string& msg) : msg_(msg) {}

std::ostream&
operator<<(std::ostream& out, const Error& err)
{
  if (!err.msg_.empty()) {
    out << err.msg_;
  }
  return out;
}

size_t
DatatypeByteSize(const std::string& dt)
{
  if (dt == "BOOL" || dt == "INT8" || dt == "UINT8" || dt == "FP8_E4M3" || dt == "FP8_E5M2") return 1;
  if (dt == "INT16" || dt == "UINT16" || dt == "FP16" || dt == "BF16") return 2;
  if (dt == "INT32" || dt == "UINT32" || dt == "FP32") return 4;
  if (dt == "INT64" || dt == "UINT64" || dt == "FP64") return 8;
  return 0;
}

//==============================================================================
Error
InferenceServerClient::ClientInferStat(InferStat* infer_stat) const
{
  std::lock_guard<std::mutex> lk(mutex_);
  *infer_stat = infer_stat_;
  return Error::Success;
}

Error
InferenceServerClient::UpdateInferStat(const RequestTimers& timer)
{
  using K = RequestTimers::Kind;
  const uint64_t request_time_ns = timer.Duration(K::REQUEST_START, K::REQUEST_END);
  const uint64_t send_time_ns = timer.Duration(K::SEND_START, K::SEND_END);
  const uint64_t recv_time_ns = timer.Duration(K::RECV_START, K::RECV_END);
  const uint64_t bad = (std::numeric_limits<uint64_t>::max)();
  if (request_time_ns == bad || send_time_ns == bad || recv_time_ns == bad) {
    return Error("Timer not set correctly." +
                 std::string(request_time_ns == bad ? " Request time from start to end is not set correctly." : "") +
                 std::string(send_time_ns == bad ? " Client send time from start to end is not set correctly." : "") +
                 std::string(recv_time_ns == bad ? " Client receive time from start to end is not set correctly." : ""));
  }
  std::lock_guard<std::mutex> lk(mutex_);
  infer_stat_.completed_request_count++;
  infer_stat_.cumulative_total_request_time_ns += request_time_ns;
  infer_stat_.cumulative_send_time_ns += send_time_ns;
  infer_stat_.cumulative_receive_time_ns += recv_time_ns;
  return Error::Success;
}

//==============================================================================
Error
InferInput::Create(
    InferInput** infer_input, const std::string& name, const std::vector<int64_t>& dims,
    const std::string& datatype)
{
  *infer_input = new InferInput(name, dims, datatype);
  return Error::Success;
}

InferInput::InferInput(const std::string& name, const std::vector<int64_t>& dims, const std::string& datatype)
    : name_(name), shape_(dims), datatype_(datatype), byte_size_(0), bufs_idx_(0), buf_pos_(0), io_type_(NONE),
      shm_offset_(0)
{
}

Error
InferInput::SetShape(const std::vector<int64_t>& shape)
{
  shape_ = shape;
  return Error::Success;
}

Error
InferInput::Reset()
{
  bufs_.clear();
  buf_byte_sizes_.clear();
  str_bufs_.clear();
  bufs_idx_ = 0;
  buf_pos_ = 0;
  byte_size_ = 0;
  io_type_ = NONE;
  shm_name_.clear();
  shm_offset_ = 0;
  return Error::Success;
}

Error
InferInput::AppendRaw(const std::vector<uint8_t>& input)
{
  return AppendRaw(input.data(), input.size());
}

Error
InferInput::AppendRaw(const uint8_t* input, size_t input_byte_size)
{
  if (io_type_ == SHARED_MEMORY) {
    return Error("The input '" + name_ + "' is already set to use shared memory; call Reset() first");
  }
  io_type_ = RAW;
  byte_size_ += input_byte_size;
  bufs_.push_back(input);
  buf_byte_sizes_.push_back(input_byte_size);
  return Error::Success;
}

Error
InferInput::SetSharedMemory(const std::string& name, size_t byte_size, size_t offset)
{
  if (io_type_ == RAW) {
    return Error("The input '" + name_ + "' already has raw data; call Reset() first");
  }
  io_type_ = SHARED_MEMORY;
  shm_name_ = name;
  byte_size_ = byte_size;
  shm_offset_ = offset;
  return Error::Success;
}

Error
InferInput::SharedMemoryInfo(std::string* name, size_t* byte_size, size_t* offset) const
{
  if (io_type_ != SHARED_MEMORY) {
    return Error("The input '" + name_ + "' is not using shared memory");
  }
  *name = shm_name_;
  *byte_size = byte_size_;
  *offset = shm_offset_;
  return Error::Success;
}

Error
InferInput::AppendFromString(const std::vector<std::string>& input)
{
  // one owned buffer holding every element as <u32 LE len><bytes>
  size_t total = 0;
  for (const auto& s : input) total += 4 + s.size();
  str_bufs_.emplace_back();
  std::string& sbuf = str_bufs_.back();
  sbuf.reserve(total);
  for (const auto& s : input) {
    const uint32_t len = static_cast<uint32_t>(s.size());
    char b[4] = {static_cast<char>(len & 0xff), static_cast<char>((len >> 8) & 0xff),
                 static_cast<char>((len >> 16) & 0xff), static_cast<char>((len >> 24) & 0xff)};
    sbuf.append(b, 4);
    sbuf.append(s);
  }
  return AppendRaw(reinterpret_cast<const uint8_t*>(sbuf.data()), sbuf.size());
}

Error
InferInput::RawData(const uint8_t** buf, size_t* byte_size)
{
  // Like the reference (common.cc:185-197) only the first buffer is returned;
  // callers needing all data should use Buffers().
  if (bufs_.empty()) {
    *buf = nullptr;
    *byte_size = 0;
  } else {
    *buf = bufs_[0];
    *byte_size = buf_byte_sizes_[0];
  }
  return Error::Success;
}

Error
InferInput::ByteSize(size_t* byte_size) const
{
  *byte_size = byte_size_;
  return Error::Success;
}

Error
InferInput::SetBinaryData(const bool binary_data)
{
  binary_data_ = binary_data;
  return Error::Success;
}

Error
InferInput::PrepareForRequest()
{
  bufs_idx_ = 0;
  buf_pos_ = 0;
  return Error::Success;
}

Error
InferInput::GetNext(uint8_t* buf, size_t size, size_t* input_bytes, bool* end_of_input)
{
  size_t copied = 0;
  while (size > 0 && bufs_idx_ < bufs_.size()) {
    const size_t left = buf_byte_sizes_[bufs_idx_] - buf_pos_;
    const size_t n = left < size ? left : size;
    std::memcpy(buf + copied, bufs_[bufs_idx_] + buf_pos_, n);
    copied += n;
    size -= n;
    buf_pos_ += n;
    if (buf_pos_ == buf_byte_sizes_[bufs_idx_]) {
      ++bufs_idx_;
      buf_pos_ = 0;
    }
  }
  *input_bytes = copied;
  *end_of_input = bufs_idx_ >= bufs_.size();
  return Error::Success;
}

Error
InferInput::GetNext(const uint8_t** buf, size_t* input_bytes, bool* end_of_input)
{
  if (bufs_idx_ < bufs_.size()) {
    *buf = bufs_[bufs_idx_] + buf_pos_;
    *input_bytes = buf_byte_sizes_[bufs_idx_] - buf_pos_;
    ++bufs_idx_;
    buf_pos_ = 0;
  } else {
    *buf = nullptr;
    *input_bytes = 0;
  }
  *end_of_input = bufs_idx_ >= bufs_.size();
  return Error::Success;
}

//==============================================================================
Error
InferRequestedOutput::Create(
    InferRequestedOutput** infer_output, const std::string& name, const size_t class_count,
    const std::string& datatype)
{
  *infer_output = new InferRequestedOutput(name, datatype, class_count);
  return Error::Success;
}

InferRequestedOutput::InferRequestedOutput(const std::string& name, const std::string& datatype, const size_t class_count)
    : name_(name), datatype_(datatype), class_count_(class_count), io_type_(NONE), shm_byte_size_(0), shm_offset_(0)
{
}

Error
InferRequestedOutput::SetSharedMemory(const std::string& region_name, const size_t byte_size, const size_t offset)
{
  if (class_count_ != 0) {
    return Error("shared memory can't be set on classification output");
  }
  io_type_ = SHARED_MEMORY;
  shm_name_ = region_name;
  shm_byte_size_ = byte_size;
  shm_offset_ = offset;
  return Error::Success;
}

Error
InferRequestedOutput::UnsetSharedMemory()
{
  io_type_ = NONE;
  shm_name_.clear();
  shm_byte_size_ = 0;
  shm_offset_ = 0;
  return Error::Success;
}

Error
InferRequestedOutput::SharedMemoryInfo(std::string* name, size_t* byte_size, size_t* offset) const
{
  if (io_type_ != SHARED_MEMORY) {
    return Error("The output '" + name_ + "' is not using shared memory");
  }
  *name = shm_name_;
  *byte_size = shm_byte_size_;
  *offset = shm_offset_;
  return Error::Success;
}

Error
InferRequestedOutput::SetBinaryData(const bool binary_data)
{
  binary_data_ = binary_data;
  return Error::Success;
}

}}  // namespace triton::client

// InferenceServerGrpcClient implementation (see include/grpc_client.h).
//
// Request marshalling mirrors reference src/c++/library/grpc_client.cc:
// 1418-1580 (parameters, shared-memory params, raw_input_contents, the
// always-present triton_enable_empty_final_response), results mirror
// InferResultGrpc (:191-446).  Unlike the reference, the request is built
// per call (the reference reuses one member ModelInferRequest and is
// therefore not thread-safe, grpc_client.h:85-90).
#include "grpc_client.h"

#include <condition_variable>
#include <cstdlib>
#include <iostream>
#include <mutex>

#include "h2.h"
#include "net.h"
#include "trace.h"

namespace triton { namespace client {

using K = RequestTimers::Kind;

namespace {

constexpr char kService[] = "/inference.GRPCInferenceService/";

GrpcCompression
ToComp(grpc_compression_algorithm a)
{
  return a == GRPC_COMPRESS_GZIP ? GrpcCompression::GZIP
         : a == GRPC_COMPRESS_DEFLATE ? GrpcCompression::DEFLATE : GrpcCompression::NONE;
}

Error
StatusToError(const GrpcStatus& st)
{
  if (st.ok()) return Error::Success;
  return Error(st.message.empty() ? st.CodeName() : st.message);
}

//------------------------------------------------------------------------------
// channel cache (reference grpc_client.cc:50-152): clients of one URL share a
// channel until TRITON_CLIENT_GRPC_CHANNEL_MAX_SHARE_COUNT (default 6) users.
struct CacheEntry {
  std::shared_ptr<H2Channel> channel;
  size_t users = 0;
};
std::mutex g_cache_mu;
std::map<std::string, std::vector<CacheEntry>> g_cache;

size_t
MaxShare()
{
  const char* e = std::getenv("TRITON_CLIENT_GRPC_CHANNEL_MAX_SHARE_COUNT");
  long v = e ? std::strtol(e, nullptr, 10) : 6;
  return v > 0 ? static_cast<size_t>(v) : 6;
}

//------------------------------------------------------------------------------
class InferResultGrpc : public InferResult {
 public:
  InferResultGrpc(std::shared_ptr<inference::ModelInferResponse> resp, Error status)
      : resp_(std::move(resp)), status_(std::move(status))
  {
    if (!resp_) return;
    const auto& outs = resp_->outputs();
    for (size_t i = 0; i < outs.size(); ++i) {
      Entry e;
      e.index = i;
      const auto& o = outs[i];
      if (i < static_cast<size_t>(resp_->raw_output_contents_size())) {
        const std::string& raw = resp_->raw_output_contents(static_cast<int>(i));
        e.data = reinterpret_cast<const uint8_t*>(raw.data());
        e.size = raw.size();
      } else if (o.has_contents()) {
        TypedToBinary(o, &e.owned);
        e.data = reinterpret_cast<const uint8_t*>(e.owned.data());
        e.size = e.owned.size();
      }
      map_.emplace(o.name(), std::move(e));
    }
    for (auto& kv : map_)
      if (!kv.second.owned.empty()) kv.second.data = reinterpret_cast<const uint8_t*>(kv.second.owned.data());
    auto it = resp_->parameters().find("triton_final_response");
    if (it != resp_->parameters().end()) {
      final_ = it->second.bool_param();
      null_ = final_ && outs.empty();
    }
  }

  Error ModelName(std::string* name) const override { *name = resp_ ? resp_->model_name() : ""; return Error::Success; }
  Error ModelVersion(std::string* v) const override { *v = resp_ ? resp_->model_version() : ""; return Error::Success; }
  Error Id(std::string* id) const override { *id = resp_ ? resp_->id() : ""; return Error::Success; }
  Error Shape(const std::string& name, std::vector<int64_t>* shape) const override
  {
    const auto* o = Out(name);
    if (!o) return Error("The response does not contain results for output name " + name);
    *shape = o->shape();
    return Error::Success;
  }
  Error Datatype(const std::string& name, std::string* dt) const override
  {
    const auto* o = Out(name);
    if (!o) return Error("The response does not contain results for output name " + name);
    *dt = o->datatype();
    return Error::Success;
  }
  Error RawData(const std::string& name, const uint8_t** buf, size_t* byte_size) const override
  {
    auto it = map_.find(name);
    if (it == map_.end()) return Error("The response does not contain results for output name " + name);
    *buf = it->second.data;
    *byte_size = it->second.size;
    return Error::Success;
  }
  Error IsFinalResponse(bool* f) const override { *f = final_; return Error::Success; }
  Error IsNullResponse(bool* n) const override { *n = null_; return Error::Success; }
  Error StringData(const std::string& name, std::vector<std::string>* out) const override
  {
    std::string dt;
    Error e = Datatype(name, &dt);
    if (!e.IsOk()) return e;
    if (dt != "BYTES") {
      return Error("This function supports tensors with datatype 'BYTES', requested output tensor '" + name +
                   "' with datatype '" + dt + "'");
    }
    const uint8_t* buf = nullptr;
    size_t n = 0;
    e = RawData(name, &buf, &n);
    if (!e.IsOk()) return e;
    out->clear();
    size_t pos = 0;
    while (pos + 4 <= n) {
      uint32_t len;
      std::memcpy(&len, buf + pos, 4);
      pos += 4;
      if (pos + len > n) return Error("malformed BYTES output '" + name + "'");
      out->emplace_back(reinterpret_cast<const char*>(buf + pos), len);
      pos += len;
    }
    return Error::Success;
  }
  std::string DebugString() const override { return resp_ ? resp_->DebugString() : std::string(); }
  Error RequestStatus() const override { return status_; }

 private:
  struct Entry {
    size_t index = 0;
    const uint8_t* data = nullptr;
    size_t size = 0;
    std::string owned;
  };
  const inference::ModelInferResponse_InferOutputTensor* Out(const std::string& name) const
  {
    if (!resp_) return nullptr;
    for (const auto& o : resp_->outputs())
      if (o.name() == name) return &o;
    return nullptr;
  }
  static void TypedToBinary(const inference::ModelInferResponse_InferOutputTensor& o, std::string* out)
  {
    const auto& c = o.contents();
    const std::string& dt = o.datatype();
    auto put = [out](const void* p, size_t n) { out->append(static_cast<const char*>(p), n); };
    if (dt == "BOOL") for (bool b : c.bool_contents()) { uint8_t x = b; put(&x, 1); }
    else if (dt == "INT8") for (int32_t v : c.int_contents()) { int8_t x = static_cast<int8_t>(v); put(&x, 1); }
    else if (dt == "INT16") for (int32_t v : c.int_contents()) { int16_t x = static_cast<int16_t>(v); put(&x, 2); }
    else if (dt == "INT32") for (int32_t v : c.int_contents()) put(&v, 4);
    else if (dt == "INT64") for (int64_t v : c.int64_contents()) put(&v, 8);
    else if (dt == "UINT8") for (uint32_t v : c.uint_contents()) { uint8_t x = static_cast<uint8_t>(v); put(&x, 1); }
    else if (dt == "UINT16") for (uint32_t v : c.uint_contents()) { uint16_t x = static_cast<uint16_t>(v); put(&x, 2); }
    else if (dt == "UINT32") for (uint32_t v : c.uint_contents()) put(&v, 4);
    else if (dt == "UINT64") for (uint64_t v : c.uint64_contents()) put(&v, 8);
    else if (dt == "FP32") for (float v : c.fp32_contents()) put(&v, 4);
    else if (dt == "FP64") for (double v : c.fp64_contents()) put(&v, 8);
    else if (dt == "BYTES")
      for (const auto& s : c.bytes_contents()) {
        uint32_t n = static_cast<uint32_t>(s.size());
        put(&n, 4);
        put(s.data(), s.size());
      }
  }

  std::shared_ptr<inference::ModelInferResponse> resp_;
  Error status_;
  std::map<std::string, Entry> map_;
  bool final_ = true;
  bool null_ = false;
};

std::vector<std::pair<std::string, std::string>>
Metadata(const Headers& h)
{
  std::vector<std::pair<std::string, std::string>> md;
  for (const auto& kv : h) md.push_back(kv);
  return md;
}

}  // namespace

//==============================================================================
InferenceServerGrpcClient::InferenceServerGrpcClient(
    const std::string& url, bool verbose, bool use_ssl, const SslOptions& ssl_options,
    const grpc::ChannelArguments& channel_args, const bool use_cached_channel, const KeepAliveOptions& keepalive)
    : InferenceServerClient(verbose), url_(url), use_cached_channel_(use_cached_channel)
{
  std::string hostport = url;
  if (hostport.compare(0, 7, "http://") == 0) hostport = hostport.substr(7);
  if (hostport.compare(0, 8, "https://") == 0) hostport = hostport.substr(8);
  size_t colon = hostport.rfind(':');
  std::string host = colon == std::string::npos ? hostport : hostport.substr(0, colon);
  int port = colon == std::string::npos ? (use_ssl ? 443 : 80) : std::atoi(hostport.c_str() + colon + 1);
  H2ChannelOptions opts;
  opts.tls.enabled = use_ssl;
  opts.tls.ca_info = ssl_options.root_certificates;
  opts.tls.cert = ssl_options.certificate_chain;
  opts.tls.key = ssl_options.private_key;
  opts.tls.alpn = "h2";
  opts.keepalive_time_ms = keepalive.keepalive_time_ms;
  opts.keepalive_timeout_ms = keepalive.keepalive_timeout_ms;
  opts.keepalive_permit_without_calls = keepalive.keepalive_permit_without_calls;
  opts.http2_max_pings_without_data = keepalive.http2_max_pings_without_data;
  for (const auto& kv : channel_args.Ints()) {
    if (kv.first == "grpc.keepalive_time_ms") opts.keepalive_time_ms = kv.second;
    if (kv.first == "grpc.keepalive_timeout_ms") opts.keepalive_timeout_ms = kv.second;
    if (kv.first == "grpc.keepalive_permit_without_calls") opts.keepalive_permit_without_calls = kv.second != 0;
    if (kv.first == "grpc.max_receive_message_length" && kv.second > 0) opts.max_message_bytes = kv.second;
  }
  // a distinct "triton_client_channel_idx" forces a private channel (reference :88-105)
  std::string idx;
  for (const auto& kv : channel_args.Ints())
    if (kv.first == "triton_client_channel_idx") idx = std::to_string(kv.second);
  cache_key_ = url + (use_ssl ? "#ssl" : "") + (idx.empty() ? "" : "#idx" + idx);
  std::string err;
  if (use_cached_channel) {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    auto& vec = g_cache[cache_key_];
    for (auto it = vec.begin(); it != vec.end();) {
      if (!it->channel->Healthy()) it = vec.erase(it);
      else ++it;
    }
    for (auto& e : vec) {
      if (e.users < MaxShare()) {
        ++e.users;
        channel_ = e.channel;
        break;
      }
    }
    if (!channel_) {
      channel_ = H2Channel::Create(host, port, opts, &err);
      if (channel_) vec.push_back({channel_, 1});
    }
  } else {
    channel_ = H2Channel::Create(host, port, opts, &err);
  }
  if (!channel_) channel_error_ = Error("failed to connect to " + url + ": " + err);
}

InferenceServerGrpcClient::~InferenceServerGrpcClient()
{
  StopStream();
  if (use_cached_channel_ && channel_) {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    auto& vec = g_cache[cache_key_];
    for (auto it = vec.begin(); it != vec.end(); ++it) {
      if (it->channel == channel_) {
        if (--it->users == 0) vec.erase(it);
        break;
      }
    }
  }
}

size_t
InferenceServerGrpcClient::GetNumCachedChannels() const
{
  std::lock_guard<std::mutex> lk(g_cache_mu);
  size_t n = 0;
  for (const auto& kv : g_cache) n += kv.second.size();
  return n;
}

Error
InferenceServerGrpcClient::Create(
    std::unique_ptr<InferenceServerGrpcClient>* client, const std::string& server_url, bool verbose, bool use_ssl,
    const SslOptions& ssl_options, const KeepAliveOptions& keepalive_options, const bool use_cached_channel)
{
  client->reset(new InferenceServerGrpcClient(server_url, verbose, use_ssl, ssl_options, grpc::ChannelArguments(),
                                              use_cached_channel, keepalive_options));
  return (*client)->channel_error_;
}

Error
InferenceServerGrpcClient::Create(
    std::unique_ptr<InferenceServerGrpcClient>* client, const std::string& server_url,
    const grpc::ChannelArguments& channel_args, bool verbose, bool use_ssl, const SslOptions& ssl_options,
    const bool use_cached_channel)
{
  client->reset(new InferenceServerGrpcClient(server_url, verbose, use_ssl, ssl_options, channel_args,
                                              use_cached_channel, KeepAliveOptions()));
  return (*client)->channel_error_;
}

Error
InferenceServerGrpcClient::UnaryRaw(
    const char* method, std::string&& request, std::string* response, const Headers& headers, uint64_t timeout_us,
    grpc_compression_algorithm comp, bool framed)
{
  if (!channel_) return channel_error_;
  struct Wait {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    GrpcStatus st;
    std::string msg;
  };
  auto w = std::make_shared<Wait>();
  H2CallHandlers h;
  h.on_message = [w](std::string&& m) { w->msg = std::move(m); };
  h.on_close = [w](const GrpcStatus& st) {
    std::lock_guard<std::mutex> lk(w->mu);
    w->st = st;
    w->done = true;
    w->cv.notify_all();
  };
  auto call = channel_->StartCall(std::string(kService) + method, Metadata(headers), timeout_us, ToComp(comp), h);
  if (framed) call->WriteFramed(std::move(request));
  else call->Write(std::move(request));
  call->WritesDone();
  std::unique_lock<std::mutex> lk(w->mu);
  w->cv.wait(lk, [&] { return w->done; });
  if (!w->st.ok()) return StatusToError(w->st);
  response->swap(w->msg);
  return Error::Success;
}

template <typename Req, typename Resp>
Error
InferenceServerGrpcClient::Unary(const char* method, const Req& request, Resp* response, const Headers& headers,
                                 uint64_t timeout_ms)
{
  std::string out;
  if (verbose_) std::cout << method << " request: " << request.DebugString() << std::endl;
  Error e = UnaryRaw(method, request.SerializeAsString(), &out, headers, timeout_ms * 1000);
  if (!e.IsOk()) return e;
  if (!response->ParseFromString(out)) return Error(std::string("failed to parse ") + method + " response");
  if (verbose_) std::cout << response->DebugString() << std::endl;
  return Error::Success;
}

Error
InferenceServerGrpcClient::IsServerLive(bool* live, const Headers& headers, const uint64_t timeout_ms)
{
  inference::ServerLiveResponse r;
  Error e = Unary("ServerLive", inference::ServerLiveRequest(), &r, headers, timeout_ms);
  *live = e.IsOk() && r.live();
  return e;
}

Error
InferenceServerGrpcClient::IsServerReady(bool* ready, const Headers& headers, const uint64_t timeout_ms)
{
  inference::ServerReadyResponse r;
  Error e = Unary("ServerReady", inference::ServerReadyRequest(), &r, headers, timeout_ms);
  *ready = e.IsOk() && r.ready();
  return e;
}

Error
InferenceServerGrpcClient::IsModelReady(
    bool* ready, const std::string& model_name, const std::string& model_version, const Headers& headers,
    const uint64_t timeout_ms)
{
  inference::ModelReadyRequest q;
  q.set_name(model_name);
  q.set_version(model_version);
  inference::ModelReadyResponse r;
  Error e = Unary("ModelReady", q, &r, headers, timeout_ms);
  *ready = e.IsOk() && r.ready();
  return e;
}

Error
InferenceServerGrpcClient::ServerMetadata(
    inference::ServerMetadataResponse* server_metadata, const Headers& headers, const uint64_t timeout_ms)
{
  return Unary("ServerMetadata", inference::ServerMetadataRequest(), server_metadata, headers, timeout_ms);
}

Error
InferenceServerGrpcClient::ModelMetadata(
    inference::ModelMetadataResponse* model_metadata, const std::string& model_name, const std::string& model_version,
    const Headers& headers, const uint64_t timeout_ms)
{
  inference::ModelMetadataRequest q;
  q.set_name(model_name);
  q.set_version(model_version);
  return Unary("ModelMetadata", q, model_metadata, headers, timeout_ms);
}

Error
InferenceServerGrpcClient::ModelConfig(
    inference::ModelConfigResponse* model_config, const std::string& model_name, const std::string& model_version,
    const Headers& headers, const uint64_t timeout_ms)
{
  inference::ModelConfigRequest q;
  q.set_name(model_name);
  q.set_version(model_version);
  return Unary("ModelConfig", q, model_config, headers, timeout_ms);
}

Error
InferenceServerGrpcClient::ModelRepositoryIndex(
    inference::RepositoryIndexResponse* repository_index, const Headers& headers, const uint64_t timeout_ms)
{
  return Unary("RepositoryIndex", inference::RepositoryIndexRequest(), repository_index, headers, timeout_ms);
}

Error
InferenceServerGrpcClient::LoadModel(
    const std::string& model_name, const Headers& headers, const std::string& config,
    const std::map<std::string, std::vector<char>>& files, const uint64_t timeout_ms)
{
  inference::RepositoryModelLoadRequest q;
  q.set_model_name(model_name);
  if (!config.empty()) (*q.mutable_parameters())["config"].set_string_param(config);
  for (const auto& kv : files) (*q.mutable_parameters())[kv.first].set_bytes_param(kv.second.data(), kv.second.size());
  inference::RepositoryModelLoadResponse r;
  return Unary("RepositoryModelLoad", q, &r, headers, timeout_ms);
}

Error
InferenceServerGrpcClient::UnloadModel(const std::string& model_name, const Headers& headers, const uint64_t timeout_ms)
{
  inference::RepositoryModelUnloadRequest q;
  q.set_model_name(model_name);
  inference::RepositoryModelUnloadResponse r;
  return Unary("RepositoryModelUnload", q, &r, headers, timeout_ms);
}

Error
InferenceServerGrpcClient::ModelInferenceStatistics(
    inference::ModelStatisticsResponse* infer_stat, const std::string& model_name, const std::string& model_version,
    const Headers& headers, const uint64_t timeout_ms)
{
  inference::ModelStatisticsRequest q;
  q.set_name(model_name);
  q.set_version(model_version);
  return Unary("ModelStatistics", q, infer_stat, headers, timeout_ms);
}

Error
InferenceServerGrpcClient::UpdateTraceSettings(
    inference::TraceSettingResponse* response, const std::string& model_name,
    const std::map<std::string, std::vector<std::string>>& settings, const Headers& headers,
    const uint64_t timeout_ms)
{
  inference::TraceSettingRequest q;
  if (!model_name.empty()) q.set_model_name(model_name);
  for (const auto& kv : settings) {
    auto& v = (*q.mutable_settings())[kv.first];
    for (const auto& s : kv.second) v.add_value(s);
  }
  return Unary("TraceSetting", q, response, headers, timeout_ms);
}

Error
InferenceServerGrpcClient::GetTraceSettings(
    inference::TraceSettingResponse* settings, const std::string& model_name, const Headers& headers,
    const uint64_t timeout_ms)
{
  inference::TraceSettingRequest q;
  if (!model_name.empty()) q.set_model_name(model_name);
  return Unary("TraceSetting", q, settings, headers, timeout_ms);
}

Error
InferenceServerGrpcClient::UpdateLogSettings(
    inference::LogSettingsResponse* response, const std::map<std::string, std::string>& settings,
    const Headers& headers, const uint64_t timeout_ms)
{
  inference::LogSettingsRequest q;
  for (const auto& kv : settings) {
    auto& v = (*q.mutable_settings())[kv.first];
    if (kv.first == "log_file" || kv.first == "log_format") v.set_string_param(kv.second);
    else if (kv.first == "log_verbose_level") v.set_uint32_param(static_cast<uint32_t>(std::stoul(kv.second)));
    else v.set_bool_param(kv.second == "true" || kv.second == "1");
  }
  return Unary("LogSettings", q, response, headers, timeout_ms);
}

Error
InferenceServerGrpcClient::GetLogSettings(inference::LogSettingsResponse* settings, const Headers& headers,
                                          const uint64_t timeout_ms)
{
  return Unary("LogSettings", inference::LogSettingsRequest(), settings, headers, timeout_ms);
}

Error
InferenceServerGrpcClient::SystemSharedMemoryStatus(
    inference::SystemSharedMemoryStatusResponse* status, const std::string& region_name, const Headers& headers,
    const uint64_t timeout_ms)
{
  inference::SystemSharedMemoryStatusRequest q;
  q.set_name(region_name);
  return Unary("SystemSharedMemoryStatus", q, status, headers, timeout_ms);
}

Error
InferenceServerGrpcClient::RegisterSystemSharedMemory(
    const std::string& name, const std::string& key, const size_t byte_size, const size_t offset,
    const Headers& headers, const uint64_t timeout_ms)
{
  inference::SystemSharedMemoryRegisterRequest q;
  q.set_name(name);
  q.set_key(key);
  q.set_offset(offset);
  q.set_byte_size(byte_size);
  inference::SystemSharedMemoryRegisterResponse r;
  return Unary("SystemSharedMemoryRegister", q, &r, headers, timeout_ms);
}

Error
InferenceServerGrpcClient::UnregisterSystemSharedMemory(const std::string& name, const Headers& headers,
                                                        const uint64_t timeout_ms)
{
  inference::SystemSharedMemoryUnregisterRequest q;
  q.set_name(name);
  inference::SystemSharedMemoryUnregisterResponse r;
  return Unary("SystemSharedMemoryUnregister", q, &r, headers, timeout_ms);
}

Error
InferenceServerGrpcClient::CudaSharedMemoryStatus(
    inference::CudaSharedMemoryStatusResponse* status, const std::string& region_name, const Headers& headers,
    const uint64_t timeout_ms)
{
  inference::CudaSharedMemoryStatusRequest q;
  q.set_name(region_name);
  return Unary("CudaSharedMemoryStatus", q, status, headers, timeout_ms);
}

Error
InferenceServerGrpcClient::RegisterCudaSharedMemory(
    const std::string& name, const cudaIpcMemHandle_t& cuda_shm_handle, const size_t device_id,
    const size_t byte_size, const Headers& headers, const uint64_t timeout_ms)
{
  inference::CudaSharedMemoryRegisterRequest q;
  q.set_name(name);
  q.set_raw_handle(reinterpret_cast<const char*>(&cuda_shm_handle), sizeof(cudaIpcMemHandle_t));
  q.set_device_id(static_cast<int64_t>(device_id));
  q.set_byte_size(byte_size);
  inference::CudaSharedMemoryRegisterResponse r;
  return Unary("CudaSharedMemoryRegister", q, &r, headers, timeout_ms);
}

Error
InferenceServerGrpcClient::UnregisterCudaSharedMemory(const std::string& name, const Headers& headers,
                                                      const uint64_t timeout_ms)
{
  inference::CudaSharedMemoryUnregisterRequest q;
  q.set_name(name);
  inference::CudaSharedMemoryUnregisterResponse r;
  return Unary("CudaSharedMemoryUnregister", q, &r, headers, timeout_ms);
}

//==============================================================================
// One-copy request encoding for uncompressed calls: the gRPC frame prefix,
// the request without its raw tensors, then every raw tensor as field 7
// (raw_input_contents) copied once from the caller's buffers — protobuf
// readers accept fields in any order.  (SerializeAsString + GrpcFrame copy
// each tensor three times.)
static void PutVarint(std::string* out, uint64_t v)
{
  while (v >= 0x80) {
    out->push_back(static_cast<char>((v & 0x7f) | 0x80));
    v >>= 7;
  }
  out->push_back(static_cast<char>(v));
}

static std::string FramedInferRequest(const inference::ModelInferRequest& head, const std::vector<InferInput*>& inputs)
{
  size_t raw = 0;
  for (InferInput* in : inputs)
    if (!in->IsSharedMemory())
      for (size_t s : in->BufferSizes()) raw += s + 16;
  std::string out;
  out.reserve(5 + 256 + raw);
  out.append(5, '\0');
  head.Encode(&out);
  for (InferInput* in : inputs) {
    if (in->IsSharedMemory()) continue;
    size_t total = 0;
    for (size_t s : in->BufferSizes()) total += s;
    out.push_back(static_cast<char>((7 << 3) | 2));
    PutVarint(&out, total);
    for (size_t i = 0; i < in->Buffers().size(); ++i)
      out.append(reinterpret_cast<const char*>(in->Buffers()[i]), in->BufferSizes()[i]);
  }
  const uint32_t n = static_cast<uint32_t>(out.size() - 5);
  out[1] = static_cast<char>(n >> 24);
  out[2] = static_cast<char>(n >> 16);
  out[3] = static_cast<char>(n >> 8);
  out[4] = static_cast<char>(n);
  return out;
}

Error
InferenceServerGrpcClient::BuildInferRequest(
    const InferOptions& options, const std::vector<InferInput*>& inputs,
    const std::vector<const InferRequestedOutput*>& outputs, inference::ModelInferRequest* req, bool include_raw)
{
  req->set_model_name(options.model_name_);
  req->set_model_version(options.model_version_);
  req->set_id(options.request_id_);
  auto& params = *req->mutable_parameters();
  params["triton_enable_empty_final_response"].set_bool_param(options.triton_enable_empty_final_response_);
  if (options.sequence_id_ != 0 || !options.sequence_id_str_.empty()) {
    if (!options.sequence_id_str_.empty()) params["sequence_id"].set_string_param(options.sequence_id_str_);
    else params["sequence_id"].set_int64_param(static_cast<int64_t>(options.sequence_id_));
    params["sequence_start"].set_bool_param(options.sequence_start_);
    params["sequence_end"].set_bool_param(options.sequence_end_);
  }
  if (options.priority_ != 0) params["priority"].set_uint64_param(options.priority_);
  if (options.server_timeout_ != 0) params["timeout"].set_int64_param(static_cast<int64_t>(options.server_timeout_));
  for (const auto& kv : options.request_parameters) {
    const RequestParameter& p = kv.second;
    if (p.name == "sequence_id" || p.name == "sequence_start" || p.name == "sequence_end" || p.name == "priority" ||
        p.name == "binary_data_output") {
      return Error("Parameter \"" + p.name + "\" is a reserved parameter and cannot be specified.");
    }
    if (p.type == "bool") params[p.name].set_bool_param(p.value == "true" || p.value == "1");
    else if (p.type == "int") params[p.name].set_int64_param(std::stoll(p.value));
    else if (p.type == "double") params[p.name].set_double_param(std::stod(p.value));
    else params[p.name].set_string_param(p.value);
  }
  for (InferInput* in : inputs) {
    auto* t = req->add_inputs();
    t->set_name(in->Name());
    t->set_datatype(in->Datatype());
    for (int64_t d : in->Shape()) t->add_shape(d);
    if (in->IsSharedMemory()) {
      std::string region;
      size_t bs, off;
      in->SharedMemoryInfo(&region, &bs, &off);
      (*t->mutable_parameters())["shared_memory_region"].set_string_param(region);
      (*t->mutable_parameters())["shared_memory_byte_size"].set_int64_param(static_cast<int64_t>(bs));
      if (off) (*t->mutable_parameters())["shared_memory_offset"].set_int64_param(static_cast<int64_t>(off));
    } else if (include_raw) {
      std::string* raw = req->add_raw_input_contents();
      size_t total = 0;
      for (size_t s : in->BufferSizes()) total += s;
      raw->reserve(total);
      for (size_t i = 0; i < in->Buffers().size(); ++i)
        raw->append(reinterpret_cast<const char*>(in->Buffers()[i]), in->BufferSizes()[i]);
    }
  }
  for (const InferRequestedOutput* o : outputs) {
    auto* t = req->add_outputs();
    t->set_name(o->Name());
    if (o->ClassificationCount() > 0)
      (*t->mutable_parameters())["classification"].set_int64_param(static_cast<int64_t>(o->ClassificationCount()));
    if (o->IsSharedMemory()) {
      std::string region;
      size_t bs, off;
      o->SharedMemoryInfo(&region, &bs, &off);
      (*t->mutable_parameters())["shared_memory_region"].set_string_param(region);
      (*t->mutable_parameters())["shared_memory_byte_size"].set_int64_param(static_cast<int64_t>(bs));
      if (off) (*t->mutable_parameters())["shared_memory_offset"].set_int64_param(static_cast<int64_t>(off));
    }
  }
  return Error::Success;
}

Error
InferenceServerGrpcClient::Infer(
    InferResult** result, const InferOptions& options, const std::vector<InferInput*>& inputs,
    const std::vector<const InferRequestedOutput*>& outputs, const Headers& headers,
    grpc_compression_algorithm compression_algorithm)
{
  trace::Range range("tc.grpc.Infer");
  RequestTimers timers;
  timers.CaptureTimestamp(K::REQUEST_START);
  timers.CaptureTimestamp(K::SEND_START);
  inference::ModelInferRequest req;
  const bool one_copy = compression_algorithm == GRPC_COMPRESS_NONE;
  Error e = BuildInferRequest(options, inputs, outputs, &req, !one_copy);
  if (!e.IsOk()) return e;
  std::string wire = one_copy ? FramedInferRequest(req, inputs) : req.SerializeAsString();
  const size_t msg_size = wire.size() - (one_copy ? 5 : 0);
  if (msg_size > static_cast<size_t>(MAX_GRPC_MESSAGE_SIZE)) {
    return Error("Request has byte size " + std::to_string(msg_size) +
                 " which exceed gRPC's byte size limit " + std::to_string(INT32_MAX) + ".");
  }
  timers.CaptureTimestamp(K::SEND_END);
  std::string out;
  e = UnaryRaw("ModelInfer", std::move(wire), &out, headers, options.client_timeout_, compression_algorithm,
               one_copy);
  timers.CaptureTimestamp(K::RECV_START);
  auto resp = std::make_shared<inference::ModelInferResponse>();
  if (e.IsOk() && !resp->ParseFromString(out)) e = Error("failed to parse ModelInferResponse");
  timers.CaptureTimestamp(K::RECV_END);
  timers.CaptureTimestamp(K::REQUEST_END);
  *result = new InferResultGrpc(e.IsOk() ? resp : nullptr, e);
  if (e.IsOk()) UpdateInferStat(timers);
  if (verbose_ && e.IsOk()) std::cout << resp->DebugString() << std::endl;
  return e;
}

Error
InferenceServerGrpcClient::AsyncInfer(
    OnCompleteFn callback, const InferOptions& options, const std::vector<InferInput*>& inputs,
    const std::vector<const InferRequestedOutput*>& outputs, const Headers& headers,
    grpc_compression_algorithm compression_algorithm)
{
  if (callback == nullptr) return Error("Callback function must be provided along with AsyncInfer() call.");
  if (!channel_) return channel_error_;
  auto timers = std::make_shared<RequestTimers>();
  timers->CaptureTimestamp(K::REQUEST_START);
  timers->CaptureTimestamp(K::SEND_START);
  inference::ModelInferRequest req;
  const bool one_copy = compression_algorithm == GRPC_COMPRESS_NONE;
  Error e = BuildInferRequest(options, inputs, outputs, &req, !one_copy);
  if (!e.IsOk()) return e;
  std::string wire = one_copy ? FramedInferRequest(req, inputs) : req.SerializeAsString();
  if (wire.size() - (one_copy ? 5 : 0) > static_cast<size_t>(MAX_GRPC_MESSAGE_SIZE))
    return Error("Request has byte size " + std::to_string(wire.size() - (one_copy ? 5 : 0)) +
                 " which exceed gRPC's byte size limit " + std::to_string(INT32_MAX) + ".");
  timers->CaptureTimestamp(K::SEND_END);
  auto msg = std::make_shared<std::string>();
  H2CallHandlers h;
  h.on_message = [msg, timers](std::string&& m) {
    timers->CaptureTimestamp(K::RECV_START);
    *msg = std::move(m);
  };
  h.on_close = [this, msg, timers, callback](const GrpcStatus& st) {
    auto resp = std::make_shared<inference::ModelInferResponse>();
    Error err = StatusToError(st);
    if (err.IsOk() && !resp->ParseFromString(*msg)) err = Error("failed to parse ModelInferResponse");
    if (timers->Timestamp(K::RECV_START) == 0) timers->CaptureTimestamp(K::RECV_START);
    timers->CaptureTimestamp(K::RECV_END);
    timers->CaptureTimestamp(K::REQUEST_END);
    if (err.IsOk()) UpdateInferStat(*timers);
    callback(new InferResultGrpc(err.IsOk() ? resp : nullptr, err));
  };
  auto call = channel_->StartCall(std::string(kService) + "ModelInfer", Metadata(headers), options.client_timeout_,
                                  ToComp(compression_algorithm), h);
  if (one_copy) call->WriteFramed(std::move(wire));
  else call->Write(std::move(wire));
  call->WritesDone();
  return Error::Success;
}

Error
InferenceServerGrpcClient::InferMulti(
    std::vector<InferResult*>* results, const std::vector<InferOptions>& options,
    const std::vector<std::vector<InferInput*>>& inputs,
    const std::vector<std::vector<const InferRequestedOutput*>>& outputs, const Headers& headers,
    grpc_compression_algorithm compression_algorithm)
{
  if (options.size() != 1 && options.size() != inputs.size())
    return Error("'options' must either contain 1 element or match size of 'inputs'");
  if (outputs.size() > 1 && outputs.size() != inputs.size())
    return Error("'outputs' must either contain 0/1 element or match size of 'inputs'");
  results->clear();
  Error first;
  static const std::vector<const InferRequestedOutput*> none;
  for (size_t i = 0; i < inputs.size(); ++i) {
    InferResult* r = nullptr;
    Error e = Infer(&r, options.size() == 1 ? options[0] : options[i], inputs[i],
                    outputs.empty() ? none : (outputs.size() == 1 ? outputs[0] : outputs[i]), headers,
                    compression_algorithm);
    if (!e.IsOk() && first.IsOk()) first = e;
    results->push_back(r);
  }
  return first;
}

Error
InferenceServerGrpcClient::AsyncInferMulti(
    OnMultiCompleteFn callback, const std::vector<InferOptions>& options,
    const std::vector<std::vector<InferInput*>>& inputs,
    const std::vector<std::vector<const InferRequestedOutput*>>& outputs, const Headers& headers,
    grpc_compression_algorithm compression_algorithm)
{
  if (callback == nullptr) return Error("Callback function must be provided along with AsyncInferMulti() call.");
  if (options.size() != 1 && options.size() != inputs.size())
    return Error("'options' must either contain 1 element or match size of 'inputs'");
  if (outputs.size() > 1 && outputs.size() != inputs.size())
    return Error("'outputs' must either contain 0/1 element or match size of 'inputs'");
  struct Fanin {
    std::atomic<size_t> left;
    std::vector<InferResult*> results;
    OnMultiCompleteFn cb;
  };
  auto st = std::make_shared<Fanin>();
  st->left = inputs.size();
  st->results.assign(inputs.size(), nullptr);
  st->cb = callback;
  static const std::vector<const InferRequestedOutput*> none;
  for (size_t i = 0; i < inputs.size(); ++i) {
    Error e = AsyncInfer(
        [st, i](InferResult* r) {
          st->results[i] = r;
          if (--st->left == 0) st->cb(st->results);
        },
        options.size() == 1 ? options[0] : options[i], inputs[i],
        outputs.empty() ? none : (outputs.size() == 1 ? outputs[0] : outputs[i]), headers, compression_algorithm);
    if (!e.IsOk()) return e;
  }
  return Error::Success;
}

//==============================================================================
Error
InferenceServerGrpcClient::StartStream(
    OnCompleteFn callback, bool enable_stats, uint32_t stream_timeout, const Headers& headers,
    grpc_compression_algorithm compression_algorithm)
{
  if (!channel_) return channel_error_;
  std::lock_guard<std::mutex> lk(stream_mutex_);
  if (stream_) {
    return Error("cannot start another stream with one already running. 'InferenceServerClient' supports only a "
                 "single active stream at a given time.");
  }
  stream_callback_ = callback;
  enable_stream_stats_ = enable_stats;
  stream_closed_ = std::make_shared<std::atomic<bool>>(false);
  auto closed = stream_closed_;
  H2CallHandlers h;
  h.on_message = [this](std::string&& m) {
    inference::ModelStreamInferResponse sr;
    std::unique_ptr<RequestTimers> timer;
    if (enable_stream_stats_) {
      std::lock_guard<std::mutex> lk2(stream_mutex_);
      if (!ongoing_stream_request_timers_.empty()) {
        timer = std::move(ongoing_stream_request_timers_.front());
        ongoing_stream_request_timers_.pop();
      }
    }
    Error err;
    std::shared_ptr<inference::ModelInferResponse> resp;
    if (!sr.ParseFromString(m)) {
      err = Error("failed to parse ModelStreamInferResponse");
    } else if (!sr.error_message().empty()) {
      err = Error(sr.error_message());
    } else {
      resp = std::make_shared<inference::ModelInferResponse>(sr.infer_response());
    }
    if (timer) {
      timer->CaptureTimestamp(K::RECV_START);
      timer->CaptureTimestamp(K::RECV_END);
      timer->CaptureTimestamp(K::REQUEST_END);
      if (err.IsOk()) UpdateInferStat(*timer);
    }
    if (stream_callback_) stream_callback_(new InferResultGrpc(resp, err));
  };
  h.on_close = [this, closed](const GrpcStatus& st) {
    if (!st.ok() && stream_callback_) stream_callback_(new InferResultGrpc(nullptr, StatusToError(st)));
    // notify under the lock: StopStream (and then the destructor) may run as
    // soon as `closed` is visible, so the cv must not be touched after unlock
    std::lock_guard<std::mutex> lk2(stream_mutex_);
    closed->store(true);
    stream_cv_.notify_all();
  };
  stream_ = channel_->StartCall(std::string(kService) + "ModelStreamInfer", Metadata(headers),
                                static_cast<uint64_t>(stream_timeout), ToComp(compression_algorithm), h);
  return Error::Success;
}

Error
InferenceServerGrpcClient::StopStream()
{
  std::shared_ptr<H2Call> s;
  std::shared_ptr<std::atomic<bool>> closed;
  {
    std::lock_guard<std::mutex> lk(stream_mutex_);
    s = stream_;
    closed = stream_closed_;
  }
  if (!s) return Error::Success;
  s->WritesDone();
  {
    std::unique_lock<std::mutex> lk(stream_mutex_);
    stream_cv_.wait(lk, [&] { return closed->load(); });
    stream_.reset();
    while (!ongoing_stream_request_timers_.empty()) ongoing_stream_request_timers_.pop();
  }
  if (verbose_) std::cout << "Stopped stream..." << std::endl;
  return Error::Success;
}

Error
InferenceServerGrpcClient::AsyncStreamInfer(
    const InferOptions& options, const std::vector<InferInput*>& inputs,
    const std::vector<const InferRequestedOutput*>& outputs)
{
  std::shared_ptr<H2Call> s;
  {
    std::lock_guard<std::mutex> lk(stream_mutex_);
    s = stream_;
  }
  if (!s) return Error("stream not available, use StartStream() to make one available.");
  std::unique_ptr<RequestTimers> timer;
  if (enable_stream_stats_) {
    timer.reset(new RequestTimers());
    timer->CaptureTimestamp(K::REQUEST_START);
    timer->CaptureTimestamp(K::SEND_START);
  }
  inference::ModelInferRequest req;
  Error e = BuildInferRequest(options, inputs, outputs, &req);
  if (!e.IsOk()) return e;
  if (timer) {
    timer->CaptureTimestamp(K::SEND_END);
    std::lock_guard<std::mutex> lk(stream_mutex_);
    ongoing_stream_request_timers_.push(std::move(timer));
  }
  s->Write(req.SerializeAsString());
  return Error::Success;
}

}}  // namespace triton::client

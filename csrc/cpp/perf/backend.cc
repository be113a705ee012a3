// perf_analyzer Backend (protocol client + control plane) and DataSet
// (request tensors, system / HIP shared-memory regions).
#include <dlfcn.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <fstream>
#include <random>
#include <sstream>

#include <hip/hip_runtime_api.h>

#include "json.h"
#include "model_config.pb.h"
#include "perf.h"
#include "shm_utils.h"

namespace tcperf {

// "REGION" or "REGION@OFFSET" (a slice of one registered region: one fan-out
// of a big region feeds every slot its own bytes)
static void SplitRegionRef(const std::string& ref, std::string* name, size_t* off)
{
  const auto at = ref.rfind('@');
  if (at == std::string::npos) {
    *name = ref;
    *off = 0;
    return;
  }
  *name = ref.substr(0, at);
  *off = static_cast<size_t>(std::stoull(ref.substr(at + 1)));
}


namespace tc = triton::client;
namespace js = triton::client::json;

uint64_t NowNs()
{
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// ============================================================================
// Backend
// ============================================================================
Error Backend::Create(const Options& o, std::unique_ptr<Backend>* out)
{
  std::unique_ptr<Backend> be(new Backend());
  be->o_ = o;
  for (const auto& kv : o.headers) be->headers_[kv.first] = kv.second;
  Error e;
  if (o.protocol == "grpc") {
    tc::SslOptions ssl;
    ssl.root_certificates = o.ssl.grpc_root_certs;
    ssl.private_key = o.ssl.grpc_private_key;
    ssl.certificate_chain = o.ssl.grpc_cert_chain;
    // a private channel per Backend: perf clients must not share one h2 connection
    e = tc::InferenceServerGrpcClient::Create(&be->grpc_, o.url, o.verbose, o.ssl.grpc_use_ssl, ssl,
                                              tc::KeepAliveOptions(), false);
  } else {
    tc::HttpSslOptions ssl;
    ssl.verify_peer = o.ssl.https_verify_peer;
    ssl.verify_host = o.ssl.https_verify_host;
    ssl.ca_info = o.ssl.https_ca;
    ssl.cert = o.ssl.https_cert;
    ssl.key = o.ssl.https_key;
    ssl.cert_type = o.ssl.https_cert_der ? tc::HttpSslOptions::CERT_DER : tc::HttpSslOptions::CERT_PEM;
    ssl.key_type = o.ssl.https_key_der ? tc::HttpSslOptions::KEY_DER : tc::HttpSslOptions::KEY_PEM;
    std::string url = o.url;
    if (o.ssl.https && url.compare(0, 8, "https://") != 0) {
      if (url.compare(0, 7, "http://") == 0) url = url.substr(7);
      url = "https://" + url;
    }
    e = tc::InferenceServerHttpClient::Create(&be->http_, url, o.verbose, ssl);
  }
  if (!e.IsOk()) return e;
  *out = std::move(be);
  return Error::Success;
}

Backend::~Backend() = default;

static std::vector<int64_t> StripBatch(std::vector<int64_t> s, int max_batch)
{
  if (max_batch > 0 && !s.empty()) s.erase(s.begin());
  return s;
}

Error Backend::ModelMeta(ModelInfo* info)
{
  *info = ModelInfo();
  if (grpc_) {
    inference::ModelConfigResponse cfg;
    Error e = grpc_->ModelConfig(&cfg, o_.model, o_.version, headers_);
    if (!e.IsOk()) return e;
    info->max_batch_size = cfg.config().max_batch_size();
    info->sequential = cfg.config().has_sequence_batching();
    info->decoupled = cfg.config().model_transaction_policy().decoupled();
    inference::ModelMetadataResponse md;
    e = grpc_->ModelMetadata(&md, o_.model, o_.version, headers_);
    if (!e.IsOk()) return e;
    for (int i = 0; i < md.inputs_size(); ++i)
      info->inputs.push_back({md.inputs(i).name(), md.inputs(i).datatype(),
                              StripBatch(md.inputs(i).shape(), info->max_batch_size)});
    for (int i = 0; i < md.outputs_size(); ++i)
      info->outputs.push_back({md.outputs(i).name(), md.outputs(i).datatype(),
                               StripBatch(md.outputs(i).shape(), info->max_batch_size)});
    return Error::Success;
  }
  std::string cfg_s, md_s, err;
  Error e = http_->ModelConfig(&cfg_s, o_.model, o_.version, headers_);
  if (!e.IsOk()) return e;
  js::Value cfg, md;
  if (!js::Parse(cfg_s, &cfg, &err)) return Error("bad model config JSON: " + err);
  if (const js::Value* v = cfg.Find("max_batch_size")) info->max_batch_size = static_cast<int>(v->AsInt());
  info->sequential = cfg.Find("sequence_batching") != nullptr;
  if (const js::Value* p = cfg.Find("model_transaction_policy"))
    if (const js::Value* d = p->Find("decoupled")) info->decoupled = d->AsBool();
  e = http_->ModelMetadata(&md_s, o_.model, o_.version, headers_);
  if (!e.IsOk()) return e;
  if (!js::Parse(md_s, &md, &err)) return Error("bad model metadata JSON: " + err);
  auto read = [&](const char* key, std::vector<TensorSpec>* out) {
    const js::Value* arr = md.Find(key);
    if (!arr) return;
    for (const auto& t : arr->Elements()) {
      TensorSpec s;
      if (const js::Value* n = t.Find("name")) s.name = n->AsString();
      if (const js::Value* d = t.Find("datatype")) s.datatype = d->AsString();
      if (const js::Value* sh = t.Find("shape"))
        for (const auto& x : sh->Elements()) s.shape.push_back(x.AsInt());
      s.shape = StripBatch(s.shape, info->max_batch_size);
      out->push_back(s);
    }
  };
  read("inputs", &info->inputs);
  read("outputs", &info->outputs);
  return Error::Success;
}

Error Backend::Stats(ServerStats* st)
{
  *st = ServerStats();
  if (grpc_) {
    inference::ModelStatisticsResponse r;
    Error e = grpc_->ModelInferenceStatistics(&r, o_.model, o_.version, headers_);
    if (!e.IsOk()) return e;
    for (int i = 0; i < r.model_stats_size(); ++i) {
      const auto& m = r.model_stats(i);
      const auto& s = m.inference_stats();
      st->inference_count += m.inference_count();
      st->execution_count += m.execution_count();
      st->success_count += s.success().count();
      st->success_ns += s.success().ns();
      st->queue_ns += s.queue().ns();
      st->compute_input_ns += s.compute_input().ns();
      st->compute_infer_ns += s.compute_infer().ns();
      st->compute_output_ns += s.compute_output().ns();
    }
    return Error::Success;
  }
  std::string s, err;
  Error e = http_->ModelInferenceStatistics(&s, o_.model, o_.version, headers_);
  if (!e.IsOk()) return e;
  js::Value v;
  if (!js::Parse(s, &v, &err)) return Error("bad statistics JSON: " + err);
  const js::Value* arr = v.Find("model_stats");
  if (!arr) return Error::Success;
  auto dur = [](const js::Value* is, const char* k, uint64_t* count, uint64_t* ns) {
    const js::Value* d = is ? is->Find(k) : nullptr;
    if (!d) return;
    if (count)
      if (const js::Value* c = d->Find("count")) *count += c->AsUInt();
    if (const js::Value* n = d->Find("ns")) *ns += n->AsUInt();
  };
  for (const auto& m : arr->Elements()) {
    if (const js::Value* x = m.Find("inference_count")) st->inference_count += x->AsUInt();
    if (const js::Value* x = m.Find("execution_count")) st->execution_count += x->AsUInt();
    const js::Value* is = m.Find("inference_stats");
    dur(is, "success", &st->success_count, &st->success_ns);
    dur(is, "queue", nullptr, &st->queue_ns);
    dur(is, "compute_input", nullptr, &st->compute_input_ns);
    dur(is, "compute_infer", nullptr, &st->compute_infer_ns);
    dur(is, "compute_output", nullptr, &st->compute_output_ns);
  }
  return Error::Success;
}

Error Backend::RegisterSystem(const std::string& name, const std::string& key, size_t bytes)
{
  return grpc_ ? grpc_->RegisterSystemSharedMemory(name, key, bytes, 0, headers_)
               : http_->RegisterSystemSharedMemory(name, key, bytes, 0, headers_);
}

Error Backend::UnregisterSystem(const std::string& name)
{
  return grpc_ ? grpc_->UnregisterSystemSharedMemory(name, headers_) : http_->UnregisterSystemSharedMemory(name, headers_);
}

Error Backend::RegisterDevice(const std::string& name, const cudaIpcMemHandle_t& h, int dev, size_t bytes)
{
  return grpc_ ? grpc_->RegisterCudaSharedMemory(name, h, dev, bytes, headers_)
               : http_->RegisterCudaSharedMemory(name, h, dev, bytes, headers_);
}

Error Backend::UnregisterDevice(const std::string& name)
{
  return grpc_ ? grpc_->UnregisterCudaSharedMemory(name, headers_) : http_->UnregisterCudaSharedMemory(name, headers_);
}

// --compression-algorithm / --grpc-compression-algorithm
static grpc_compression_algorithm GrpcCompression(const std::string& c)
{
  return c == "gzip" ? GRPC_COMPRESS_GZIP : c == "deflate" ? GRPC_COMPRESS_DEFLATE : GRPC_COMPRESS_NONE;
}

static tc::InferenceServerHttpClient::CompressionType HttpCompression(const std::string& c)
{
  using CT = tc::InferenceServerHttpClient::CompressionType;
  return c == "gzip" ? CT::GZIP : c == "deflate" ? CT::DEFLATE : CT::NONE;
}

Error Backend::AsyncInfer(std::function<void(InferResult*)> cb, const InferOptions& opt,
                          const std::vector<InferInput*>& in, const std::vector<const InferRequestedOutput*>& out)
{
  if (grpc_) return grpc_->AsyncInfer(cb, opt, in, out, headers_, GrpcCompression(o_.compression));
  const auto ct = HttpCompression(o_.compression);
  return http_->AsyncInfer(cb, opt, in, out, headers_, tc::Parameters(), ct, ct);
}

Error Backend::SyncInfer(InferResult** r, const InferOptions& opt, const std::vector<InferInput*>& in,
                         const std::vector<const InferRequestedOutput*>& out)
{
  if (grpc_) return grpc_->Infer(r, opt, in, out, headers_, GrpcCompression(o_.compression));
  const auto ct = HttpCompression(o_.compression);
  return http_->Infer(r, opt, in, out, headers_, tc::Parameters(), ct, ct);
}

Error Backend::StartStream(std::function<void(InferResult*)> cb)
{
  if (!grpc_) return Error("streaming requires gRPC");
  return grpc_->StartStream(cb, true, 0, headers_, GrpcCompression(o_.compression));
}

Error Backend::StreamInfer(const InferOptions& opt, const std::vector<InferInput*>& in,
                           const std::vector<const InferRequestedOutput*>& out)
{
  if (!grpc_) return Error("streaming requires gRPC");
  return grpc_->AsyncStreamInfer(opt, in, out);
}

Error Backend::StopStream()
{
  return grpc_ ? grpc_->StopStream() : Error::Success;
}

Error Backend::ClientStat(tc::InferStat* st)
{
  return grpc_ ? grpc_->ClientInferStat(st) : http_->ClientInferStat(st);
}

// ============================================================================
// DataSet
// ============================================================================
namespace {

size_t DtypeSize(const std::string& dt)
{
  if (dt == "BOOL" || dt == "INT8" || dt == "UINT8") return 1;
  if (dt == "INT16" || dt == "UINT16" || dt == "FP16" || dt == "BF16") return 2;
  if (dt == "INT32" || dt == "UINT32" || dt == "FP32") return 4;
  if (dt == "INT64" || dt == "UINT64" || dt == "FP64") return 8;
  return 0;  // BYTES
}

// dtype codes of csrc/kernels/common.h (K1 synth_fill)
int DtypeCode(const std::string& dt)
{
  static const std::map<std::string, int> m = {
      {"BOOL", 0}, {"INT8", 1}, {"INT16", 2}, {"INT32", 3}, {"INT64", 4}, {"UINT8", 5}, {"UINT16", 6},
      {"UINT32", 7}, {"UINT64", 8}, {"FP16", 9}, {"FP32", 10}, {"FP64", 11}, {"BF16", 12}};
  auto it = m.find(dt);
  return it == m.end() ? -1 : it->second;
}

// IEEE fp32 -> fp16 bits, round to nearest even (host compilers without _Float16)
uint16_t F32ToF16(float f)
{
  uint32_t x;
  memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  const int32_t exp = static_cast<int32_t>((x >> 23) & 0xff) - 127 + 15;
  uint32_t mant = x & 0x7fffffu;
  if (((x >> 23) & 0xff) == 0xff) return static_cast<uint16_t>(sign | 0x7c00u | (mant ? 0x200u : 0));
  if (exp >= 31) return static_cast<uint16_t>(sign | 0x7c00u);
  if (exp <= 0) {
    if (exp < -10) return static_cast<uint16_t>(sign);
    mant |= 0x800000u;
    const int shift = 14 - exp;
    uint32_t h = mant >> shift;
    const uint32_t rem = mant & ((1u << shift) - 1), half = 1u << (shift - 1);
    if (rem > half || (rem == half && (h & 1))) ++h;
    return static_cast<uint16_t>(sign | h);
  }
  uint32_t h = (static_cast<uint32_t>(exp) << 10) | (mant >> 13);
  const uint32_t rem = mant & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1))) ++h;
  return static_cast<uint16_t>(sign | h);
}

int64_t Elements(const std::vector<int64_t>& s)
{
  int64_t n = 1;
  for (auto d : s) n *= d;
  return n;
}

typedef int (*SynthFillFn)(void*, size_t, int, int, double, double, uint64_t, uint64_t, void*);
typedef int (*PackBytesFn)(const void*, const uint32_t*, uint64_t, void*, void*, void*);
typedef uint64_t (*PackBytesWsFn)(uint64_t);
typedef int (*ConvertFn)(const void*, int, void*, int, size_t, int, void*);

bool NarrowFloat(const std::string& dt) { return dt == "FP16" || dt == "BF16"; }

// host fallback of K4/K5: BF16 by truncation (the wire format of the
// reference's serialize_bf16_tensor), FP16 round-to-nearest-even
void NarrowOnHost(const std::string& dt, const std::vector<float>& f, std::vector<uint8_t>* out)
{
  out->resize(f.size() * 2);
  for (size_t i = 0; i < f.size(); ++i) {
    uint16_t h;
    if (dt == "BF16") {
      uint32_t u;
      memcpy(&u, &f[i], 4);
      h = static_cast<uint16_t>(u >> 16);
    } else {
      h = F32ToF16(f[i]);
    }
    memcpy(out->data() + 2 * i, &h, 2);
  }
}

// K1/K2 live in the framework's libtcamd_hip.so; find it next to this
// binary's tree (csrc/cpp/build/{bin,lib} -> triton_client_amd/ops/lib) or via
// $TCAMD_HIP_LIB.
void* HipKernelLib()
{
  static void* handle = []() -> void* {
    std::vector<std::string> cands;
    if (const char* env = getenv("TCAMD_HIP_LIB")) cands.push_back(env);
    Dl_info info;
    if (dladdr(reinterpret_cast<void*>(&HipKernelLib), &info) && info.dli_fname) {
      std::string p = info.dli_fname;
      auto slash = p.rfind('/');
      std::string dir = slash == std::string::npos ? "." : p.substr(0, slash);
      cands.push_back(dir + "/../../../../triton_client_amd/ops/lib/libtcamd_hip.so");
    }
    for (const auto& c : cands)
      if (void* h = dlopen(c.c_str(), RTLD_NOW | RTLD_GLOBAL)) return h;
    return nullptr;
  }();
  return handle;
}

template <typename F>
F HipKernel(const char* sym)
{
  void* h = HipKernelLib();
  return h ? reinterpret_cast<F>(dlsym(h, sym)) : nullptr;
}

}  // namespace

DataSet::~DataSet()
{
  for (auto& v : inputs_)
    for (auto* i : v) delete i;
  if (stream_) (void)hipStreamDestroy(static_cast<hipStream_t>(stream_));
  for (auto& v : outputs_)
    for (auto* o : v) delete o;
}

const std::vector<const InferRequestedOutput*>& DataSet::Outputs(size_t slot) const
{
  return outputs_c_[slot % outputs_c_.size()];
}

Error DataSet::MakeRegion(Backend* be, const std::string& name, size_t bytes, bool device, Region* r)
{
  r->name = name;
  r->bytes = bytes;
  r->device = device;
  if (device) {
    hipError_t he = hipSetDevice(o_.device);
    if (he == hipSuccess) he = hipMalloc(&r->dev, bytes);
    if (he != hipSuccess) return Error(std::string("hipMalloc failed: ") + hipGetErrorString(he));
    he = hipMemset(r->dev, 0, bytes);
    cudaIpcMemHandle_t h;
    if (he == hipSuccess) he = hipIpcGetMemHandle(&h, r->dev);
    if (he != hipSuccess) return Error(std::string("hipIpcGetMemHandle failed: ") + hipGetErrorString(he));
    return be->RegisterDevice(name, h, o_.device, bytes);
  }
  r->key = "/tcperf_" + std::to_string(getpid()) + "_" + name;
  Error e = tc::CreateSharedMemoryRegion(r->key, bytes, &r->fd);
  if (!e.IsOk()) return e;
  e = tc::MapSharedMemory(r->fd, 0, bytes, &r->host);
  if (!e.IsOk()) return e;
  return be->RegisterSystem(name, r->key, bytes);
}

Error DataSet::FillHost(const TensorSpec& t, const std::vector<int64_t>& shape, std::vector<uint8_t>* bytes,
                        std::vector<std::string>* strs)
{
  const int64_t n = Elements(shape);  // the whole batch: every element drawn, not one sample replicated
  std::mt19937_64 rng(o_.seed * 1000003ull + std::hash<std::string>()(t.name));
  if (t.datatype == "BYTES") {
    strs->clear();
    for (int64_t i = 0; i < n; ++i) {
      if (!o_.string_data.empty()) {
        strs->push_back(o_.string_data);
      } else if (o_.input_data == "zero") {
        strs->push_back(std::string(o_.string_length, '0'));
      } else {
        std::string s(o_.string_length, ' ');
        for (auto& c : s) c = static_cast<char>('a' + rng() % 26);
        strs->push_back(s);
      }
    }
    return Error::Success;
  }
  const size_t es = DtypeSize(t.datatype);
  if (es == 0) return Error("unsupported datatype " + t.datatype + " for input " + t.name);
  bytes->assign(n * es, 0);
  if (o_.input_data == "zero") return Error::Success;
  std::uniform_real_distribution<float> uf(0.f, 1.f);
  for (int64_t i = 0; i < n; ++i) {
    uint8_t* p = bytes->data() + i * es;
    const std::string& dt = t.datatype;
    if (dt == "FP32") {
      float v = uf(rng);
      memcpy(p, &v, 4);
    } else if (dt == "FP64") {
      double v = uf(rng);
      memcpy(p, &v, 8);
    } else if (dt == "FP16") {
      const uint16_t v = F32ToF16(uf(rng));
      memcpy(p, &v, 2);
    } else if (dt == "BF16") {
      float v = uf(rng);
      uint32_t u;
      memcpy(&u, &v, 4);
      uint16_t h = static_cast<uint16_t>(u >> 16);
      memcpy(p, &h, 2);
    } else if (dt == "BOOL") {
      p[0] = rng() & 1;
    } else {
      uint64_t v = rng() % 100;  // small non-negative ints are valid for every int type
      memcpy(p, &v, es);
    }
  }
  return Error::Success;
}

static Error LoadJsonData(const std::string& path, std::vector<js::Value>* entries)
{
  std::ifstream f(path);
  if (!f) return Error("cannot open --input-data file " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  js::Value v;
  std::string err;
  if (!js::Parse(ss.str(), &v, &err)) return Error("bad --input-data JSON: " + err);
  const js::Value* d = v.Find("data");
  if (!d || !d->IsArray() || d->Size() == 0) return Error("--input-data JSON needs a non-empty \"data\" array");
  // perf_analyzer's layout: "data": [ {step 0}, {step 1}, ... ] (a nested
  // array per stream is flattened: every request cycles through all steps)
  for (const auto& e : d->Elements()) {
    if (e.IsArray())
      for (const auto& x : e.Elements()) entries->push_back(x);
    else
      entries->push_back(e);
  }
  return Error::Success;
}

Error DataSet::Init(const Options& o, const ModelInfo& info, Backend* be, size_t max_slots, bool fill_inputs)
{
  o_ = o;
  {
    static std::atomic<int> seq{0};
    const int n = seq.fetch_add(1);
    prefix_ = n == 0 ? std::string("perf_") : "perf" + std::to_string(getpid()) + "_" + std::to_string(n) + "_";
  }
  const bool shm = o.shared_memory != "none";
  const bool dev = o.shared_memory == "hip";
  const bool json_data = o.input_data != "random" && o.input_data != "zero";
  std::vector<js::Value> entries;
  if (json_data) {
    Error e = LoadJsonData(o.input_data, &entries);
    if (!e.IsOk()) return e;
  }
  size_t n_entries = json_data ? entries.size() : 1;
  for (const auto& kv : o.preregistered_input_lists) n_entries = std::max(n_entries, kv.second.size());
  slot_entries_ = !o.preregistered_input_lists.empty();
  const int bs = info.max_batch_size > 0 ? o.batch : 1;
  if (info.max_batch_size == 0 && o.batch > 1) return Error("model does not support batching; use -b 1");
  if (info.max_batch_size > 0 && o.batch > info.max_batch_size)
    return Error("batch " + std::to_string(o.batch) + " exceeds max_batch_size " +
                 std::to_string(info.max_batch_size));
  hipStream_t st = nullptr;
  if (dev) {
    hipError_t he = hipSetDevice(o.device);
    if (he == hipSuccess) he = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (he != hipSuccess) return Error(std::string("hipStreamCreate failed: ") + hipGetErrorString(he));
    stream_ = st;
  }
  std::ostringstream desc;
  bool used_k1 = false, used_k2 = false, used_k4 = false;
  inputs_.resize(n_entries);
  for (size_t ent = 0; ent < n_entries; ++ent) {
    for (const auto& t : info.inputs) {
      std::vector<int64_t> shape = t.shape;
      auto so = o.shapes.find(t.name);
      if (so != o.shapes.end()) shape = so->second;
      for (auto d : shape)
        if (d < 0) return Error("input " + t.name + " has a variable dim; pass --shape " + t.name + ":...");
      std::vector<int64_t> full = shape;
      if (info.max_batch_size > 0) full.insert(full.begin(), bs);
      InferInput* in;
      Error e = InferInput::Create(&in, t.name, full, t.datatype);
      if (!e.IsOk()) return e;
      inputs_[ent].push_back(in);
      if (o.input_tensor_format == "json") {
        e = in->SetBinaryData(false);  // HTTP: the tensor goes as an inline JSON "data" array
        if (!e.IsOk()) return e;
      }
      const std::string rname = prefix_ + "in_" + t.name + (ent ? "_e" + std::to_string(ent) : std::string());

      // device-synthesised data (HIP shm, random): K1 numeric fill, or K1
      // characters + K2 length-prefixed packing for BYTES; nothing is built
      // on the host and the batch is NOT one sample replicated
      const bool k1_numeric = dev && !json_data && t.datatype != "BYTES" && o.input_data == "random";
      const bool k2_bytes = dev && !json_data && t.datatype == "BYTES" && o.string_data.empty();
      if ((k1_numeric || k2_bytes) && !o.preregistered_inputs.count(t.name)) {
        const int64_t n = Elements(full);
        const size_t bytes = k2_bytes ? static_cast<size_t>(n) * (4 + o.string_length)
                                      : static_cast<size_t>(n) * DtypeSize(t.datatype);
        Region r;
        e = MakeRegion(be, rname, bytes, true, &r);
        regions_.push_back(r);
        input_regions_.push_back(regions_.size() - 1);
        if (!e.IsOk()) return e;
        if (fill_inputs) {
          auto k1 = HipKernel<SynthFillFn>("tcamd_synth_fill");
          if (!k1) return Error("HIP shm synthetic data needs K1 (tcamd_synth_fill in libtcamd_hip.so)");
          int rc = 0;
          if (k1_numeric) {
            const bool fp = t.datatype == "FP32" || t.datatype == "FP16" || t.datatype == "BF16" || t.datatype == "FP64";
            rc = k1(r.dev, n, DtypeCode(t.datatype), 2 /*uniform*/, 0.0, fp ? 1.0 : 100.0, o.seed, ent, st);
          } else {
            auto k2 = HipKernel<PackBytesFn>("tcamd_pack_bytes");
            auto k2ws = HipKernel<PackBytesWsFn>("tcamd_pack_bytes_workspace");
            if (!k2 || !k2ws) return Error("HIP shm BYTES data needs K2 (tcamd_pack_bytes in libtcamd_hip.so)");
            // chars: K1 uniform u8 in ['a', 'a'+26) ('0' for zero data); lens: K1 constant
            const size_t chars = static_cast<size_t>(n) * o.string_length;
            void *payload = nullptr, *lens = nullptr, *ws = nullptr;
            const uint64_t wsb = k2ws(n);
            hipError_t he = hipMallocAsync(&payload, std::max<size_t>(16, chars), st);
            if (he == hipSuccess) he = hipMallocAsync(&lens, 4 * static_cast<size_t>(n), st);
            if (he == hipSuccess) he = hipMallocAsync(&ws, wsb, st);
            if (he != hipSuccess) return Error(std::string("hipMallocAsync failed: ") + hipGetErrorString(he));
            if (o.input_data == "zero") rc = k1(payload, chars, DtypeCode("UINT8"), 1 /*const*/, '0', 0, o.seed, ent, st);
            else rc = k1(payload, chars, DtypeCode("UINT8"), 2 /*uniform*/, 'a', 'a' + 26, o.seed, ent, st);
            if (rc == 0) rc = k1(lens, n, DtypeCode("UINT32"), 1 /*const*/, o.string_length, 0, 0, 0, st);
            if (rc == 0) rc = k2(payload, static_cast<const uint32_t*>(lens), n, r.dev, ws, st);
            (void)hipFreeAsync(payload, st);
            (void)hipFreeAsync(lens, st);
            (void)hipFreeAsync(ws, st);
            used_k2 = true;
          }
          if (rc == 0) rc = hipStreamSynchronize(st);
          if (rc != 0) return Error("device synthetic fill failed: " + std::to_string(rc));
          used_k1 = true;
        }
        in->SetSharedMemory(r.name, r.bytes, 0);
        continue;
      }

      // host-built data: JSON content, or random/zero without HIP shm
      std::vector<uint8_t> sample;
      std::vector<std::string> strs;
      std::vector<float> narrow;  // JSON FP16/BF16 values, narrowed by K4/K5 on the device (HIP shm)
      if (json_data) {
        const js::Value& jd = entries[ent];
        const js::Value* v = jd.Find(t.name);
        if (!v) return Error("--input-data JSON has no entry for input " + t.name);
        const js::Value* content = v->IsObject() ? v->Find("content") : v;
        if (v->IsObject())
          if (const js::Value* sh = v->Find("shape")) {
            shape.clear();
            for (const auto& x : sh->Elements()) shape.push_back(x.AsInt());
            full = shape;
            if (info.max_batch_size > 0) full.insert(full.begin(), bs);
            in->SetShape(full);
          }
        if (!content || !content->IsArray()) return Error("--input-data: bad content for " + t.name);
        const size_t es = DtypeSize(t.datatype);
        for (const auto& x : content->Elements()) {
          if (t.datatype == "BYTES") {
            strs.push_back(x.AsString());
            continue;
          }
          if (NarrowFloat(t.datatype)) {
            narrow.push_back(static_cast<float>(x.AsDouble()));
            continue;
          }
          uint8_t buf[8] = {0};
          if (t.datatype == "FP32") { float f = static_cast<float>(x.AsDouble()); memcpy(buf, &f, 4); }
          else if (t.datatype == "FP64") { double f = x.AsDouble(); memcpy(buf, &f, 8); }
          else if (t.datatype == "BOOL") { buf[0] = x.AsBool() ? 1 : 0; }
          else { int64_t iv = x.AsInt(); memcpy(buf, &iv, es); }
          sample.insert(sample.end(), buf, buf + es);
        }
        if (NarrowFloat(t.datatype)) {
          if (static_cast<int64_t>(narrow.size()) != Elements(shape))
            return Error("--input-data: element count of " + t.name + " does not match its shape");
          if (!(dev && fill_inputs)) NarrowOnHost(t.datatype, narrow, &sample);
          else sample.assign(narrow.size() * es, 0);  // sized here, written on the device below
        }
        if (t.datatype != "BYTES" && static_cast<int64_t>(sample.size()) != Elements(shape) * (int64_t)es)
          return Error("--input-data: element count of " + t.name + " does not match its shape");
      } else {
        // the whole batch (JSON content is one sample: replicated below)
        e = FillHost(t, full, &sample, &strs);
        if (!e.IsOk()) return e;
      }
      const int reps = json_data ? bs : 1;
      std::vector<uint8_t> batch_bytes;
      if (t.datatype == "BYTES") {
        for (int b = 0; b < reps; ++b)
          for (const auto& s : strs) {
            uint32_t len = static_cast<uint32_t>(s.size());
            const uint8_t* lp = reinterpret_cast<const uint8_t*>(&len);
            batch_bytes.insert(batch_bytes.end(), lp, lp + 4);
            batch_bytes.insert(batch_bytes.end(), s.begin(), s.end());
          }
      } else {
        for (int b = 0; b < reps; ++b) batch_bytes.insert(batch_bytes.end(), sample.begin(), sample.end());
      }
      if (!shm) {
        host_data_.push_back(std::move(batch_bytes));
        in->AppendRaw(host_data_.back().data(), host_data_.back().size());
        continue;
      }
      auto pre = o.preregistered_inputs.find(t.name);
      if (pre != o.preregistered_inputs.end()) {
        auto lst = o.preregistered_input_lists.find(t.name);
        if (lst != o.preregistered_input_lists.end()) {
          std::string rn;
          size_t off = 0;
          SplitRegionRef(lst->second[ent % lst->second.size()], &rn, &off);
          in->SetSharedMemory(rn, batch_bytes.size(), off);
          if (ent == 0) desc << t.name << ": " << lst->second.size() << " caller regions pinned to slots; ";
          continue;
        }
        in->SetSharedMemory(pre->second, batch_bytes.size(), 0);
        if (ent == 0) desc << t.name << ": caller region '" << pre->second << "'; ";
        continue;
      }
      Region r;
      e = MakeRegion(be, rname, batch_bytes.size(), dev, &r);
      regions_.push_back(r);
      input_regions_.push_back(regions_.size() - 1);
      if (!e.IsOk()) return e;
      if (fill_inputs) {
        if (dev && !narrow.empty()) {
          // K4/K5: the JSON values go up as fp32 once per batch row and are
          // narrowed straight into the region (BF16 truncation = the wire format)
          auto cvt = HipKernel<ConvertFn>("tcamd_convert");
          if (!cvt) return Error("HIP shm FP16/BF16 JSON data needs K4/K5 (tcamd_convert in libtcamd_hip.so)");
          std::vector<float> rows;
          for (int b = 0; b < reps; ++b) rows.insert(rows.end(), narrow.begin(), narrow.end());
          void* tmp = nullptr;
          hipError_t he = hipMallocAsync(&tmp, std::max<size_t>(16, rows.size() * 4), st);
          if (he == hipSuccess) he = hipMemcpyAsync(tmp, rows.data(), rows.size() * 4, hipMemcpyHostToDevice, st);
          int rc = he == hipSuccess ? cvt(tmp, DtypeCode("FP32"), r.dev, DtypeCode(t.datatype), rows.size(), 0, st) : he;
          (void)hipFreeAsync(tmp, st);
          if (rc == 0) rc = hipStreamSynchronize(st);
          if (rc != 0) return Error("device FP16/BF16 conversion failed: " + std::to_string(rc));
          used_k4 = true;
        } else if (dev) {
          hipError_t he = hipMemcpyAsync(r.dev, batch_bytes.data(), batch_bytes.size(), hipMemcpyHostToDevice, st);
          if (he == hipSuccess) he = hipStreamSynchronize(st);
          if (he != hipSuccess) return Error(std::string("hipMemcpy failed: ") + hipGetErrorString(he));
        } else {
          memcpy(r.host, batch_bytes.data(), batch_bytes.size());
        }
      }
      in->SetSharedMemory(r.name, r.bytes, 0);
    }
  }
  // outputs: one region per slot per output in shm mode
  const size_t nslot = shm ? std::max<size_t>(1, max_slots) : 1;
  outputs_.resize(nslot);
  outputs_c_.resize(nslot);
  for (size_t s = 0; s < nslot; ++s) {
    for (const auto& t : info.outputs) {
      InferRequestedOutput* out;
      Error e = InferRequestedOutput::Create(&out, t.name);
      if (!e.IsOk()) return e;
      if (o.output_tensor_format == "json" && !shm) {
        e = out->SetBinaryData(false);
        if (!e.IsOk()) return e;
      }
      outputs_[s].push_back(out);
      outputs_c_[s].push_back(out);
      if (!shm) continue;
      size_t bytes = o.output_shm_size;
      const size_t es = DtypeSize(t.datatype);
      bool fixed = es > 0;
      for (auto d : t.shape) fixed = fixed && d >= 0;
      if (fixed) bytes = std::max<size_t>(bytes, static_cast<size_t>(Elements(t.shape)) * es * bs);
      auto po = o.preregistered_outputs.find(t.name);
      if (po != o.preregistered_outputs.end()) {
        // a caller region: the output's exact size when the shape is fixed
        // (the server checks it against the region), else --output-shared-memory-size
        const size_t exact = fixed ? static_cast<size_t>(Elements(t.shape)) * es * bs : o.output_shm_size;
        std::string rn;
        size_t off = 0;
        SplitRegionRef(po->second[s % po->second.size()], &rn, &off);
        out->SetSharedMemory(rn, exact, off);
        continue;
      }
      Region r;
      e = MakeRegion(be, prefix_ + "out_" + t.name + "_" + std::to_string(s), bytes, dev, &r);
      regions_.push_back(r);
      if (!e.IsOk()) return e;
      out->SetSharedMemory(r.name, r.bytes, 0);
    }
  }
  std::ostringstream d2;
  d2 << (json_data ? "json:" + o.input_data : o.input_data) << " data";
  if (n_entries > 1) d2 << " (" << n_entries << " entries, cycled per request)";
  d2 << ", ";
  d2 << (shm ? (dev ? "HIP shared memory (device " + std::to_string(o.device) + ")" : std::string("system shared memory"))
             : std::string("in-band tensors"));
  if (used_k1) d2 << ", inputs filled on device by K1 Philox (seed " << o.seed << ")";
  if (used_k2) d2 << " + K2 BYTES packing";
  if (used_k4) d2 << ", JSON FP16/BF16 values narrowed on device by K4/K5";
  if (o.input_tensor_format == "json" || o.output_tensor_format == "json")
    d2 << ", tensors in/out as " << o.input_tensor_format << "/" << o.output_tensor_format;
  if (o.compression != "none") d2 << ", " << o.compression << " compression";
  if (!o.request_parameters.empty()) d2 << ", " << o.request_parameters.size() << " request parameter(s)";
  if (!fill_inputs && !input_regions_.empty()) d2 << ", inputs replicated by fan-out";
  if (!desc.str().empty()) d2 << "; " << desc.str();
  describe_ = d2.str();
  return Error::Success;
}

std::vector<DataSet::RegionView> DataSet::InputRegions() const
{
  std::vector<RegionView> v;
  for (size_t i : input_regions_) {
    const Region& r = regions_[i];
    v.push_back({r.device ? r.dev : r.host, r.bytes, r.device, o_.device});
  }
  return v;
}

void DataSet::Release(Backend* be)
{
  for (auto& r : regions_) {
    if (be) {
      if (r.device) be->UnregisterDevice(r.name);
      else be->UnregisterSystem(r.name);
    }
    if (r.device && r.dev) (void)hipFree(r.dev);
    if (!r.device) {
      if (r.host) tc::UnmapSharedMemory(r.host, r.bytes);
      if (r.fd >= 0) tc::CloseSharedMemory(r.fd);
      if (!r.key.empty()) tc::UnlinkSharedMemoryRegion(r.key);
    }
  }
  regions_.clear();
}

}  // namespace tcperf

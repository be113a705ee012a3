// C++ client test-suite (port of the scenarios in reference
// src/c++/tests/cc_client_test.cc, client_timeout_test.cc and the C++
// examples), run against the in-repo KServe-v2 server:
//
//   cc_client_test <http host:port> <grpc host:port>
//
// Every test runs for BOTH InferenceServerHttpClient and
// InferenceServerGrpcClient where the API exists on both (the reference's
// typed gtest suite).  No gtest on the box: a tiny CHECK harness instead.
#include <unistd.h>

// white-box access through the C10 friend hook (see include/common.h)
#define TRITON_INFERENCE_SERVER_CLIENT_CLASS InternalsProbe

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <iostream>
#include <memory>
#include <mutex>
#include <thread>

#include "grpc_client.h"
#include "http_client.h"
#include "json.h"
#include "shm_utils.h"

namespace tc = triton::client;

namespace triton { namespace client {
// Granted friendship by TRITON_INFERENCE_SERVER_CLIENT_CLASS.
class InternalsProbe {
 public:
  static size_t BufferCount(const InferInput* in) { return in->bufs_.size(); }
  static size_t StringBufferCount(const InferInput* in) { return in->str_bufs_.size(); }
  static bool IsShm(const InferInput* in) { return in->io_type_ == InferInput::SHARED_MEMORY; }
  static size_t ByteSize(const InferInput* in) { return in->byte_size_; }
  static size_t ShmOffset(const InferRequestedOutput* out) { return out->shm_offset_; }
};
}}  // namespace triton::client

static int g_failures = 0;
static int g_checks = 0;
#define CHECK(cond, msg)                                                                        \
  do {                                                                                         \
    ++g_checks;                                                                                \
    if (!(cond)) {                                                                             \
      ++g_failures;                                                                            \
      std::cerr << "  FAILED " << __FILE__ << ":" << __LINE__ << ": " << #cond << " -- " << msg \
                << std::endl;                                                                  \
    }                                                                                          \
  } while (0)
#define CHECK_OK(err, what) CHECK((err).IsOk(), what << ": " << (err).Message())

static std::string g_http, g_grpc;

struct Tensors {
  std::vector<int32_t> in0, in1;
  std::unique_ptr<tc::InferInput> i0, i1;
  std::vector<tc::InferInput*> inputs;
  Tensors()
  {
    for (int i = 0; i < 16; ++i) {
      in0.push_back(i);
      in1.push_back(1);
    }
    tc::InferInput *a, *b;
    tc::InferInput::Create(&a, "INPUT0", {1, 16}, "INT32");
    tc::InferInput::Create(&b, "INPUT1", {1, 16}, "INT32");
    i0.reset(a);
    i1.reset(b);
    i0->AppendRaw(reinterpret_cast<uint8_t*>(in0.data()), 64);
    i1->AppendRaw(reinterpret_cast<uint8_t*>(in1.data()), 64);
    inputs = {i0.get(), i1.get()};
  }
};

static void
CheckAddSub(tc::InferResult* r, bool swapped, const std::string& ctx)
{
  CHECK_OK(r->RequestStatus(), ctx);
  const uint8_t* b0;
  size_t n0;
  const uint8_t* b1;
  size_t n1;
  CHECK_OK(r->RawData("OUTPUT0", &b0, &n0), ctx);
  CHECK_OK(r->RawData("OUTPUT1", &b1, &n1), ctx);
  if (n0 != 64 || n1 != 64) {
    CHECK(false, ctx << " wrong output byte size " << n0 << "/" << n1);
    return;
  }
  // HTTP outputs sit right after the JSON header, at any byte offset: copy
  // out instead of reading int32 through a misaligned pointer (UBSan)
  int32_t o0[16], o1[16];
  std::memcpy(o0, b0, sizeof(o0));
  std::memcpy(o1, b1, sizeof(o1));
  for (int i = 0; i < 16; ++i) {
    int sum = i + 1, diff = i - 1;
    CHECK(o0[i] == (swapped ? diff : sum), ctx << " OUTPUT0[" << i << "]=" << o0[i]);
    CHECK(o1[i] == (swapped ? sum : diff), ctx << " OUTPUT1[" << i << "]=" << o1[i]);
  }
  std::vector<int64_t> shape;
  CHECK_OK(r->Shape("OUTPUT0", &shape), ctx);
  CHECK(shape.size() == 2 && shape[1] == 16, ctx << " shape");
  std::string dt;
  r->Datatype("OUTPUT0", &dt);
  CHECK(dt == "INT32", ctx << " datatype " << dt);
}

// ---------------------------------------------------------------------------
template <typename Client>
void
TestHealthAndMetadata(Client* c, const std::string& kind)
{
  bool live = false, ready = false, mready = false, bad = true;
  CHECK_OK(c->IsServerLive(&live), kind);
  CHECK_OK(c->IsServerReady(&ready), kind);
  CHECK(live && ready, kind << " live/ready");
  c->IsModelReady(&mready, "simple");
  CHECK(mready, kind << " simple ready");
  c->IsModelReady(&bad, "no_such_model");
  CHECK(!bad, kind << " unknown model must not be ready");
}

template <typename Client>
void
TestInfer(Client* c, const std::string& kind)
{
  Tensors t;
  tc::InferOptions opt("simple");
  opt.request_id_ = "cc-1";
  tc::InferResult* r = nullptr;
  CHECK_OK(c->Infer(&r, opt, t.inputs), kind << " Infer");
  if (r) {
    CheckAddSub(r, false, kind + " Infer");
    std::string id;
    r->Id(&id);
    CHECK(id == "cc-1", kind << " id " << id);
    delete r;
  }
  // explicit outputs
  tc::InferRequestedOutput *o0, *o1;
  tc::InferRequestedOutput::Create(&o0, "OUTPUT0");
  tc::InferRequestedOutput::Create(&o1, "OUTPUT1");
  std::unique_ptr<tc::InferRequestedOutput> u0(o0), u1(o1);
  CHECK_OK(c->Infer(&r, opt, t.inputs, {o0, o1}), kind << " Infer with outputs");
  if (r) {
    CheckAddSub(r, false, kind + " Infer outputs");
    delete r;
  }
}

template <typename Client>
void
TestAsyncAndMulti(Client* c, const std::string& kind)
{
  Tensors t;
  std::mutex mu;
  std::condition_variable cv;
  int done = 0;
  const int N = 32;
  for (int i = 0; i < N; ++i) {
    tc::InferOptions opt("simple");
    CHECK_OK(c->AsyncInfer(
                 [&](tc::InferResult* r) {
                   CheckAddSub(r, false, kind + " AsyncInfer");
                   delete r;
                   std::lock_guard<std::mutex> lk(mu);
                   ++done;
                   cv.notify_all();
                 },
                 opt, t.inputs),
             kind << " AsyncInfer");
  }
  {
    std::unique_lock<std::mutex> lk(mu);
    bool ok = cv.wait_for(lk, std::chrono::seconds(30), [&] { return done == N; });
    CHECK(ok, kind << " async completions " << done);
  }
  // InferMulti over versions 1..3 of onnx_int32_int32_int32 (v2/v3 swap outputs)
  std::vector<tc::InferOptions> opts;
  std::vector<std::vector<tc::InferInput*>> ins;
  for (int v = 1; v <= 3; ++v) {
    opts.emplace_back("onnx_int32_int32_int32");
    opts.back().model_version_ = std::to_string(v);
    ins.push_back(t.inputs);
  }
  std::vector<tc::InferResult*> results;
  CHECK_OK(c->InferMulti(&results, opts, ins), kind << " InferMulti");
  for (size_t i = 0; i < results.size(); ++i) {
    CheckAddSub(results[i], i != 0, kind + " InferMulti v" + std::to_string(i + 1));
    delete results[i];
  }
  // AsyncInferMulti
  std::atomic<bool> multi_done{false};
  CHECK_OK(c->AsyncInferMulti(
               [&](std::vector<tc::InferResult*> rs) {
                 for (size_t i = 0; i < rs.size(); ++i) {
                   CheckAddSub(rs[i], i != 0, kind + " AsyncInferMulti");
                   delete rs[i];
                 }
                 multi_done = true;
               },
               opts, ins),
           kind << " AsyncInferMulti");
  for (int i = 0; i < 300 && !multi_done; ++i) usleep(10000);
  CHECK(multi_done, kind << " AsyncInferMulti completion");
  tc::InferStat st;
  c->ClientInferStat(&st);
  CHECK(st.completed_request_count >= 36, kind << " stats count " << st.completed_request_count);
}

template <typename Client>
void
TestStrings(Client* c, const std::string& kind)
{
  tc::InferInput *a, *b;
  tc::InferInput::Create(&a, "INPUT0", {1, 16}, "BYTES");
  tc::InferInput::Create(&b, "INPUT1", {1, 16}, "BYTES");
  std::unique_ptr<tc::InferInput> ua(a), ub(b);
  std::vector<std::string> s0, s1;
  for (int i = 0; i < 16; ++i) {
    s0.push_back(std::to_string(i));
    s1.push_back("1");
  }
  a->AppendFromString(s0);
  b->AppendFromString(s1);
  tc::InferResult* r = nullptr;
  CHECK_OK(c->Infer(&r, tc::InferOptions("simple_string"), {a, b}), kind << " string infer");
  if (r) {
    std::vector<std::string> out;
    CHECK_OK(r->StringData("OUTPUT0", &out), kind << " StringData");
    CHECK(out.size() == 16 && out[5] == "6", kind << " string result");
    delete r;
  }
}

template <typename Client>
void
TestSystemShm(Client* c, const std::string& kind)
{
  std::string key = "/cc_test_" + kind;
  int fd;
  CHECK_OK(tc::CreateSharedMemoryRegion(key, 256, &fd), kind << " shm create");
  void* addr;
  CHECK_OK(tc::MapSharedMemory(fd, 0, 256, &addr), kind << " shm map");
  int32_t* p = static_cast<int32_t*>(addr);
  for (int i = 0; i < 16; ++i) {
    p[i] = i;
    p[16 + i] = 1;
  }
  CHECK_OK(c->RegisterSystemSharedMemory("cc_shm_" + kind, key, 256), kind << " register");
  tc::InferInput *a, *b;
  tc::InferInput::Create(&a, "INPUT0", {1, 16}, "INT32");
  tc::InferInput::Create(&b, "INPUT1", {1, 16}, "INT32");
  std::unique_ptr<tc::InferInput> ua(a), ub(b);
  a->SetSharedMemory("cc_shm_" + kind, 64, 0);
  b->SetSharedMemory("cc_shm_" + kind, 64, 64);
  tc::InferRequestedOutput *o0, *o1;
  tc::InferRequestedOutput::Create(&o0, "OUTPUT0");
  tc::InferRequestedOutput::Create(&o1, "OUTPUT1");
  std::unique_ptr<tc::InferRequestedOutput> u0(o0), u1(o1);
  o0->SetSharedMemory("cc_shm_" + kind, 64, 128);
  o1->SetSharedMemory("cc_shm_" + kind, 64, 192);
  tc::InferResult* r = nullptr;
  CHECK_OK(c->Infer(&r, tc::InferOptions("simple"), {a, b}, {o0, o1}), kind << " shm infer");
  delete r;
  for (int i = 0; i < 16; ++i) {
    CHECK(p[32 + i] == i + 1 && p[48 + i] == i - 1, kind << " shm output " << i);
  }
  CHECK_OK(c->UnregisterSystemSharedMemory("cc_shm_" + kind), kind << " unregister");
  tc::UnmapSharedMemory(addr, 256);
  tc::CloseSharedMemory(fd);
  tc::UnlinkSharedMemoryRegion(key);
}

// HTTP's LoadModel takes query params before the config (reference
// http_client.h vs grpc_client.h); dispatch like the reference test fixture.
tc::Error
Load(tc::InferenceServerHttpClient* c, const std::string& name, const std::string& config,
     const std::map<std::string, std::vector<char>>& files = {})
{
  return c->LoadModel(name, tc::Headers(), tc::Parameters(), config, files);
}
tc::Error
Load(tc::InferenceServerGrpcClient* c, const std::string& name, const std::string& config,
     const std::map<std::string, std::vector<char>>& files = {})
{
  return c->LoadModel(name, tc::Headers(), config, files);
}

template <typename Client>
void
TestLoadOverride(Client* c, const std::string& kind)
{
  const std::string name = "onnx_int32_int32_int32";
  tc::Error e = Load(c, name, "{\"backend\":\"onnxruntime\", not json");
  CHECK(!e.IsOk(), kind << " malformed config must fail");
  bool r3 = false;
  c->IsModelReady(&r3, name, "3");
  CHECK(r3, kind << " v3 still ready after failed load");
  CHECK_OK(Load(c, name, "{\"backend\":\"onnxruntime\",\"version_policy\":{\"specific\":{\"versions\":[2]}}}"),
           kind << " config override");
  bool r2 = false;
  c->IsModelReady(&r2, name, "2");
  c->IsModelReady(&r3, name, "3");
  CHECK(r2 && !r3, kind << " only v2 after override");
  std::string content = "tcamd-model:onnx_int32_int32_int32";
  std::map<std::string, std::vector<char>> files{{"file:1/model.onnx", std::vector<char>(content.begin(), content.end())}};
  e = Load(c, name, "", files);
  CHECK(!e.IsOk(), kind << " files without config must fail");
  std::string ovr = "cc_override_" + kind;
  CHECK_OK(Load(c, ovr, "{\"backend\":\"onnxruntime\"}", files), kind << " file override");
  bool ro = false;
  c->IsModelReady(&ro, ovr, "1");
  CHECK(ro, kind << " override v1 ready");
  CHECK_OK(c->UnloadModel(ovr), kind << " unload override");
  CHECK_OK(Load(c, name, "{\"backend\":\"onnxruntime\",\"version_policy\":{\"all\":{}}}"),
           kind << " restore all versions");
}

template <typename Client>
void
TestTimeout(Client* c, const std::string& kind)
{
  std::vector<int32_t> d(4, 7);
  tc::InferInput* a;
  tc::InferInput::Create(&a, "INPUT0", {1, 4}, "INT32");
  std::unique_ptr<tc::InferInput> ua(a);
  a->AppendRaw(reinterpret_cast<uint8_t*>(d.data()), 16);
  tc::InferOptions opt("custom_identity_int32");
  opt.client_timeout_ = 50000;  // 50 ms vs a 500 ms model
  tc::InferResult* r = nullptr;
  tc::Error e = c->Infer(&r, opt, {a});
  CHECK(!e.IsOk() && e.Message().find("Deadline") != std::string::npos, kind << " timeout: " << e.Message());
  delete r;
  opt.client_timeout_ = 0;
  e = c->Infer(&r, opt, {a});
  CHECK_OK(e, kind << " no timeout");
  delete r;
}

// ---------------------------------------------------------------------------
void
TestGrpcSpecific(tc::InferenceServerGrpcClient* c)
{
  inference::ServerMetadataResponse md;
  CHECK_OK(c->ServerMetadata(&md), "grpc ServerMetadata");
  CHECK(md.name() == "triton-mi355x", "grpc server name " << md.name());
  inference::ModelConfigResponse cfg;
  CHECK_OK(c->ModelConfig(&cfg, "simple"), "grpc ModelConfig");
  CHECK(cfg.config().max_batch_size() == 8, "grpc max_batch_size");
  inference::ModelStatisticsResponse st;
  CHECK_OK(c->ModelInferenceStatistics(&st, "simple"), "grpc stats");
  CHECK(st.model_stats_size() == 1 && st.model_stats(0).inference_count() > 0, "grpc stats content");
  inference::TraceSettingResponse tr;
  CHECK_OK(c->UpdateTraceSettings(&tr, "simple", {{"trace_rate", {"7"}}}), "grpc trace update");
  auto it = tr.settings().find("trace_rate");
  CHECK(it != tr.settings().end() && it->second.value_size() == 1 && it->second.value(0) == "7", "grpc trace value");
  CHECK_OK(c->UpdateTraceSettings(&tr, "simple", {{"trace_rate", {}}}), "grpc trace clear");
  inference::RepositoryIndexResponse idx;
  CHECK_OK(c->ModelRepositoryIndex(&idx), "grpc index");
  CHECK(idx.models_size() > 5, "grpc index size");

  // bidirectional stream: two interleaved sequences on simple_sequence
  std::mutex mu;
  std::condition_variable cv;
  std::map<std::string, std::vector<int>> got;
  int received = 0;
  CHECK_OK(c->StartStream([&](tc::InferResult* r) {
             std::lock_guard<std::mutex> lk(mu);
             if (r->RequestStatus().IsOk()) {
               std::string id;
               r->Id(&id);
               const uint8_t* b;
               size_t n;
               if (r->RawData("OUTPUT", &b, &n).IsOk() && n == 4) got[id.substr(0, 4)].push_back(*reinterpret_cast<const int32_t*>(b));
             }
             ++received;
             delete r;
             cv.notify_all();
           }),
           "grpc StartStream");
  std::vector<int> values = {0, 11, 7, 5, 3, 2, 0, 1};
  std::vector<std::unique_ptr<tc::InferInput>> keep;
  std::vector<std::vector<int32_t>> data;
  data.reserve(2 * values.size());
  for (size_t s = 0; s < values.size(); ++s) {
    for (int seq = 0; seq < 2; ++seq) {
      data.push_back({seq == 0 ? values[s] : -values[s] + (s == 0 ? 100 : 0)});
      tc::InferInput* in;
      tc::InferInput::Create(&in, "INPUT", {1, 1}, "INT32");
      in->AppendRaw(reinterpret_cast<uint8_t*>(data.back().data()), 4);
      keep.emplace_back(in);
      tc::InferOptions o("simple_sequence");
      o.sequence_id_ = 1000 + seq;
      o.sequence_start_ = s == 0;
      o.sequence_end_ = s + 1 == values.size();
      o.request_id_ = std::to_string(1000 + seq) + "_" + std::to_string(s);
      CHECK_OK(c->AsyncStreamInfer(o, {in}), "grpc AsyncStreamInfer");
    }
  }
  {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait_for(lk, std::chrono::seconds(20), [&] { return received >= 16; });
  }
  CHECK(got["1000"].size() == values.size(), "seq 1000 responses " << got["1000"].size());
  if (got["1000"].size() == values.size()) {
    CHECK(got["1000"][0] == 1, "seq start adds 1");
    for (size_t s = 1; s < values.size(); ++s) CHECK(got["1000"][s] == values[s], "seq value " << s);
    CHECK(got["1001"][0] == 101, "seq1 start");
  }
  // decoupled repeat_int32 with empty final response
  received = 0;
  std::vector<int32_t> in_v = {4, 5, 6};
  std::vector<uint32_t> delay_v = {1, 1, 1};
  std::vector<uint32_t> wait_v = {0};
  tc::InferInput *i_in, *i_delay, *i_wait;
  tc::InferInput::Create(&i_in, "IN", {3}, "INT32");
  tc::InferInput::Create(&i_delay, "DELAY", {3}, "UINT32");
  tc::InferInput::Create(&i_wait, "WAIT", {1}, "UINT32");
  keep.emplace_back(i_in);
  keep.emplace_back(i_delay);
  keep.emplace_back(i_wait);
  i_in->AppendRaw(reinterpret_cast<uint8_t*>(in_v.data()), 12);
  i_delay->AppendRaw(reinterpret_cast<uint8_t*>(delay_v.data()), 12);
  i_wait->AppendRaw(reinterpret_cast<uint8_t*>(wait_v.data()), 4);
  tc::InferOptions ro("repeat_int32");
  ro.triton_enable_empty_final_response_ = true;
  CHECK_OK(c->AsyncStreamInfer(ro, {i_in, i_delay, i_wait}), "grpc decoupled");
  {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait_for(lk, std::chrono::seconds(20), [&] { return received >= 4; });
  }
  CHECK(received == 4, "decoupled responses (3 + empty final) " << received);
  CHECK_OK(c->StopStream(), "grpc StopStream");
  CHECK(c->GetNumCachedChannels() >= 1, "channel cache");
}

void
TestHttpSpecific(tc::InferenceServerHttpClient* c)
{
  std::string md;
  CHECK_OK(c->ServerMetadata(&md), "http ServerMetadata");
  CHECK(md.find("triton-mi355x") != std::string::npos, "http metadata " << md);
  std::string cfg;
  CHECK_OK(c->ModelConfig(&cfg, "simple"), "http ModelConfig");
  CHECK(cfg.find("\"max_batch_size\":8") != std::string::npos, "http config " << cfg);
  std::string trace;
  CHECK_OK(c->UpdateTraceSettings(&trace, "simple", {{"trace_rate", {"9"}}}), "http trace update");
  CHECK(trace.find("\"trace_rate\":\"9\"") != std::string::npos, "http trace " << trace);
  CHECK_OK(c->UpdateTraceSettings(&trace, "simple", {{"trace_rate", {}}}), "http trace clear");
  // compression + JSON (non-binary) tensors
  Tensors t;
  t.i1->SetBinaryData(false);
  tc::InferRequestedOutput* o;
  tc::InferRequestedOutput::Create(&o, "OUTPUT0");
  std::unique_ptr<tc::InferRequestedOutput> uo(o);
  o->SetBinaryData(false);
  tc::InferResult* r = nullptr;
  CHECK_OK(c->Infer(&r, tc::InferOptions("simple"), t.inputs, {o}, tc::Headers(), tc::Parameters(),
                    tc::InferenceServerHttpClient::CompressionType::GZIP,
                    tc::InferenceServerHttpClient::CompressionType::DEFLATE),
           "http compressed JSON infer");
  if (r) {
    const uint8_t* b;
    size_t n;
    CHECK_OK(r->RawData("OUTPUT0", &b, &n), "json output as binary");
    CHECK(n == 64 && reinterpret_cast<const int32_t*>(b)[3] == 4, "json output value");
    delete r;
  }
  // GenerateRequestBody / ParseResponseBody round trip
  std::vector<char> body;
  size_t hl = 0;
  Tensors t2;
  CHECK_OK(tc::InferenceServerHttpClient::GenerateRequestBody(&body, &hl, tc::InferOptions("simple"), t2.inputs),
           "GenerateRequestBody");
  CHECK(hl > 0 && body.size() == hl + 128, "request body size " << body.size());
  std::string resp = "{\"model_name\":\"m\",\"outputs\":[{\"name\":\"o\",\"datatype\":\"FP64\",\"shape\":[2],\"data\":[1.5,2.5]}]}";
  tc::InferResult* pr = nullptr;
  CHECK_OK(tc::InferenceServerHttpClient::ParseResponseBody(&pr, std::vector<char>(resp.begin(), resp.end())),
           "ParseResponseBody");
  if (pr) {
    const uint8_t* b;
    size_t n;
    CHECK_OK(pr->RawData("o", &b, &n), "parsed FP64 json output");
    CHECK(n == 16 && reinterpret_cast<const double*>(b)[1] == 2.5, "FP64 JSON->binary (no overflow)");
    delete pr;
  }
  std::string logs;
  CHECK_OK(c->UpdateLogSettings(&logs, {{"log_verbose_level", "1"}}), "http log settings");
  CHECK(logs.find("\"log_verbose_level\":1") != std::string::npos, "log settings " << logs);
}

// Binary <-> JSON data conversion for every datatype, both directions, plus
// the invalid cases (behaviour matrix of reference
// src/c++/tests/cc_client_test.cc:1641-2171, exercised through the public
// GenerateRequestBody / ParseResponseBody entry points; no server).
namespace js = triton::client::json;

template <typename T>
static std::vector<uint8_t>
Bytes(std::initializer_list<T> v)
{
  std::vector<uint8_t> b(v.size() * sizeof(T));
  std::memcpy(b.data(), std::data(v), b.size());
  return b;
}

// input (two AppendRaw chunks, sent as JSON) -> the request header's data array
static bool
InputJsonData(const std::string& dt, const std::vector<uint8_t>& a, const std::vector<uint8_t>& b, int64_t n,
              js::Value* data, std::string* err)
{
  tc::InferInput* in;
  tc::InferInput::Create(&in, "INPUT", {n}, dt);
  std::unique_ptr<tc::InferInput> own(in);
  in->AppendRaw(a);
  in->AppendRaw(b);
  in->SetBinaryData(false);
  std::vector<char> body;
  size_t hl = 0;
  tc::Error e = tc::InferenceServerHttpClient::GenerateRequestBody(&body, &hl, tc::InferOptions("m"), {in});
  if (!e.IsOk()) {
    *err = e.Message();
    return false;
  }
  js::Value root;
  if (!js::Parse(body.data(), hl, &root, err)) return false;
  const js::Value* ins = root.Find("inputs");
  if (!ins || ins->Size() != 1) return false;
  const js::Value* d = (*ins)[0].Find("data");
  if (!d || ((*ins)[0].Find("parameters") && (*ins)[0].Find("parameters")->Find("binary_data_size"))) return false;
  *data = *d;
  return body.size() == hl;  // nothing sent in the binary section
}

// JSON output (a response body) -> the binary the result hands out
static bool
OutputBinary(const std::string& dt, const std::string& json_data, size_t n, std::vector<uint8_t>* out)
{
  std::string resp = "{\"model_name\":\"m\",\"outputs\":[{\"name\":\"o\",\"datatype\":\"" + dt + "\",\"shape\":[" +
                     std::to_string(n) + "],\"data\":" + json_data + "}]}";
  tc::InferResult* r = nullptr;
  tc::Error e = tc::InferenceServerHttpClient::ParseResponseBody(&r, std::vector<char>(resp.begin(), resp.end()));
  std::unique_ptr<tc::InferResult> own(r);
  if (!e.IsOk() || !r || !r->RequestStatus().IsOk()) return false;
  const uint8_t* b;
  size_t sz;
  if (!r->RawData("o", &b, &sz).IsOk()) return false;
  out->assign(b, b + sz);
  return true;
}

static void
TestJsonDataMatrix()
{
  js::Value d;
  std::string err;
  // input -> JSON: the two appended chunks flatten into one array, in order
  CHECK(InputJsonData("INT32", Bytes<int32_t>({1, 3, 5, 7}), Bytes<int32_t>({2, 4, 6, 8}), 8, &d, &err), err);
  CHECK(d.Size() == 8 && d[0].AsInt() == 1 && d[3].AsInt() == 7 && d[4].AsInt() == 2 && d[7].AsInt() == 8,
        "flattened AppendRaw chain");
  struct Case {
    const char* dt;
    std::vector<uint8_t> a, b;
    std::function<bool(const js::Value&)> check;
  };
  const std::vector<Case> cases = {
      {"BOOL", Bytes<uint8_t>({0}), Bytes<uint8_t>({1}),
       [](const js::Value& v) { return v[0].type() == js::Value::Type::Bool && !v[0].AsBool() && v[1].AsBool(); }},
      {"UINT8", Bytes<uint8_t>({1}), Bytes<uint8_t>({UINT8_MAX}),
       [](const js::Value& v) { return v[0].AsUInt() == 1 && v[1].AsUInt() == UINT8_MAX; }},
      {"UINT16", Bytes<uint16_t>({1}), Bytes<uint16_t>({UINT16_MAX}),
       [](const js::Value& v) { return v[0].AsUInt() == 1 && v[1].AsUInt() == UINT16_MAX; }},
      {"UINT32", Bytes<uint32_t>({1}), Bytes<uint32_t>({UINT32_MAX}),
       [](const js::Value& v) { return v[0].AsUInt() == 1 && v[1].AsUInt() == UINT32_MAX; }},
      {"UINT64", Bytes<uint64_t>({1}), Bytes<uint64_t>({UINT64_MAX}),
       [](const js::Value& v) { return v[0].AsUInt() == 1 && v[1].AsUInt() == UINT64_MAX; }},
      {"INT8", Bytes<int8_t>({INT8_MIN}), Bytes<int8_t>({INT8_MAX}),
       [](const js::Value& v) { return v[0].AsInt() == INT8_MIN && v[1].AsInt() == INT8_MAX; }},
      {"INT16", Bytes<int16_t>({INT16_MIN}), Bytes<int16_t>({INT16_MAX}),
       [](const js::Value& v) { return v[0].AsInt() == INT16_MIN && v[1].AsInt() == INT16_MAX; }},
      {"INT32", Bytes<int32_t>({INT32_MIN}), Bytes<int32_t>({INT32_MAX}),
       [](const js::Value& v) { return v[0].AsInt() == INT32_MIN && v[1].AsInt() == INT32_MAX; }},
      {"INT64", Bytes<int64_t>({INT64_MIN}), Bytes<int64_t>({INT64_MAX}),
       [](const js::Value& v) { return v[0].AsInt() == INT64_MIN && v[1].AsInt() == INT64_MAX; }},
      {"FP32", Bytes<float>({-1.5f}), Bytes<float>({3.25e7f}),
       [](const js::Value& v) { return v[0].AsDouble() == -1.5 && (float)v[1].AsDouble() == 3.25e7f; }},
      {"FP64", Bytes<double>({-0.125}), Bytes<double>({1e300}),
       [](const js::Value& v) { return v[0].AsDouble() == -0.125 && v[1].AsDouble() == 1e300; }},
  };
  for (const auto& c : cases) {
    const bool ok = InputJsonData(c.dt, c.a, c.b, 2, &d, &err);
    CHECK(ok && d.Size() == 2 && c.check(d), "input " << c.dt << " -> JSON " << err);
  }
  // BYTES: two length-prefixed elements in separate chunks -> two JSON strings
  {
    std::vector<uint8_t> a = {2, 0, 0, 0, 'a', 'b'}, b = {3, 0, 0, 0, 'c', 'd', 'e'};
    const bool ok = InputJsonData("BYTES", a, b, 2, &d, &err);
    CHECK(ok && d.Size() == 2 && d[0].AsString() == "ab" && d[1].AsString() == "cde", "input BYTES -> JSON " << err);
  }
  // invalid: half/bfloat16/fp8 cannot be JSON numbers; unknown datatypes fail
  for (const char* bad : {"FP16", "BF16", "FP8_E4M3", "invaliddatatype"})
    CHECK(!InputJsonData(bad, Bytes<uint16_t>({1}), Bytes<uint16_t>({2}), 2, &d, &err), "input " << bad << " must fail");

  // JSON -> binary (response data arrays)
  std::vector<uint8_t> out;
  auto same = [&](const std::vector<uint8_t>& want) { return out == want; };
  CHECK(OutputBinary("BOOL", "[false,true]", 2, &out) && same({0, 1}), "output BOOL");
  CHECK(OutputBinary("UINT8", "[1,255]", 2, &out) && same(Bytes<uint8_t>({1, 255})), "output UINT8");
  CHECK(OutputBinary("UINT16", "[1,65535]", 2, &out) && same(Bytes<uint16_t>({1, 65535})), "output UINT16");
  CHECK(OutputBinary("UINT32", "[1,4294967295]", 2, &out) && same(Bytes<uint32_t>({1, 4294967295u})),
        "output UINT32");
  CHECK(OutputBinary("UINT64", "[1,18446744073709551615]", 2, &out) && same(Bytes<uint64_t>({1, UINT64_MAX})),
        "output UINT64");
  CHECK(OutputBinary("INT8", "[-128,127]", 2, &out) && same(Bytes<int8_t>({-128, 127})), "output INT8");
  CHECK(OutputBinary("INT16", "[-32768,32767]", 2, &out) && same(Bytes<int16_t>({-32768, 32767})), "output INT16");
  CHECK(OutputBinary("INT32", "[-2147483648,2147483647]", 2, &out) && same(Bytes<int32_t>({INT32_MIN, INT32_MAX})),
        "output INT32");
  CHECK(OutputBinary("INT64", "[-9223372036854775808,9223372036854775807]", 2, &out) &&
            same(Bytes<int64_t>({INT64_MIN, INT64_MAX})),
        "output INT64");
  CHECK(OutputBinary("FP32", "[-1.5,3.25e7]", 2, &out) && same(Bytes<float>({-1.5f, 3.25e7f})), "output FP32");
  CHECK(OutputBinary("FP64", "[-0.125,1e300]", 2, &out) && same(Bytes<double>({-0.125, 1e300})), "output FP64");
  CHECK(OutputBinary("INT32", "[[1,2],[3,4]]", 4, &out) && same(Bytes<int32_t>({1, 2, 3, 4})),
        "nested JSON arrays flatten row-major");
  CHECK(OutputBinary("BYTES", "[\"ab\",\"\"]", 2, &out) && same({2, 0, 0, 0, 'a', 'b', 0, 0, 0, 0}), "output BYTES");
  for (const char* bad : {"FP16", "BF16", "invaliddatatype"})
    CHECK(!OutputBinary(bad, "[1,2]", 2, &out), "output " << bad << " must fail");
}

// InferInput buffer chain state, through the friend hook (reference
// src/c++/tests/cc_client_test.cc:29-33 uses the same mechanism).
static void
TestFriendHook()
{
  using P = tc::InternalsProbe;
  tc::InferInput* in;
  CHECK_OK(tc::InferInput::Create(&in, "X", {1, 4}, "INT32"), "create");
  std::unique_ptr<tc::InferInput> own(in);
  std::vector<uint8_t> a(8), b(8);
  CHECK_OK(in->AppendRaw(a), "append a");
  CHECK_OK(in->AppendRaw(b), "append b");
  CHECK(P::BufferCount(in) == 2 && P::ByteSize(in) == 16, "two buffers, 16 bytes");
  CHECK_OK(in->Reset(), "reset");
  CHECK(P::BufferCount(in) == 0 && P::ByteSize(in) == 0, "reset clears the chain");
  CHECK_OK(in->SetSharedMemory("r", 16, 0), "shm");
  CHECK(P::IsShm(in) && P::BufferCount(in) == 0, "shm input has no buffers");
  tc::InferInput* s;
  CHECK_OK(tc::InferInput::Create(&s, "S", {2}, "BYTES"), "create bytes");
  std::unique_ptr<tc::InferInput> own_s(s);
  CHECK_OK(s->AppendFromString({"ab", "cde"}), "append strings");
  CHECK(P::StringBufferCount(s) == 1 && P::ByteSize(s) == 4 + 2 + 4 + 3, "strings owned by the input");
  tc::InferRequestedOutput* o;
  CHECK_OK(tc::InferRequestedOutput::Create(&o, "Y"), "output");
  std::unique_ptr<tc::InferRequestedOutput> own_o(o);
  CHECK_OK(o->SetSharedMemory("r", 64, 32), "output shm");
  CHECK(P::ShmOffset(o) == 32, "output shm offset");
}

int
main(int argc, char** argv)
{
  g_http = argc > 1 ? argv[1] : "localhost:8000";
  g_grpc = argc > 2 ? argv[2] : "localhost:8001";
  std::unique_ptr<tc::InferenceServerHttpClient> http;
  std::unique_ptr<tc::InferenceServerGrpcClient> grpc;
  CHECK_OK(tc::InferenceServerHttpClient::Create(&http, g_http), "http create");
  CHECK_OK(tc::InferenceServerGrpcClient::Create(&grpc, g_grpc), "grpc create");
  if (g_failures) return 1;
  struct T {
    const char* name;
    std::function<void()> fn;
  };
  std::vector<T> tests = {
      {"friend hook", [&] { TestFriendHook(); }},
      {"json data matrix", [&] { TestJsonDataMatrix(); }},
      {"health/metadata", [&] { TestHealthAndMetadata(http.get(), "http"); TestHealthAndMetadata(grpc.get(), "grpc"); }},
      {"infer", [&] { TestInfer(http.get(), "http"); TestInfer(grpc.get(), "grpc"); }},
      {"async/multi", [&] { TestAsyncAndMulti(http.get(), "http"); TestAsyncAndMulti(grpc.get(), "grpc"); }},
      {"strings", [&] { TestStrings(http.get(), "http"); TestStrings(grpc.get(), "grpc"); }},
      {"system shm", [&] { TestSystemShm(http.get(), "http"); TestSystemShm(grpc.get(), "grpc"); }},
      {"load overrides", [&] { TestLoadOverride(http.get(), "http"); TestLoadOverride(grpc.get(), "grpc"); }},
      {"timeouts", [&] { TestTimeout(http.get(), "http"); TestTimeout(grpc.get(), "grpc"); }},
      {"http specific", [&] { TestHttpSpecific(http.get()); }},
      {"grpc specific", [&] { TestGrpcSpecific(grpc.get()); }},
  };
  for (auto& t : tests) {
    int before = g_failures;
    t.fn();
    std::cout << (g_failures == before ? "[ PASS ] " : "[ FAIL ] ") << t.name << std::endl;
  }
  std::cout << g_checks << " checks, " << g_failures << " failures" << std::endl;
  return g_failures ? 1 : 0;
}

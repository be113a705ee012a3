// client_timeout_test: every client-side deadline path of the C++ clients
// (behavioral parity with reference src/c++/tests/client_timeout_test.cc,
// same CLI): sync / async (HTTP, gRPC) and streaming (gRPC) inference with
// InferOptions::client_timeout_ against the slow `custom_identity_int32`
// model, and (-p, gRPC) every control-plane RPC with its timeout_ms.
//
//   client_timeout_test [-v] [-i http|grpc] [-u url] [-a] [-s] [-t timeout] [-p] [-H k:v]
//
// -t is the client timeout: microseconds for inference (InferOptions), and
// the same number as milliseconds for the -p control calls, as in the
// reference.  Exit 0 = every call succeeded; any error (e.g. "Deadline
// Exceeded") is printed and exits 1, which is what the harness checks.
// -H adds a request header; our test server honours `tc-fault-delay-ms`
// to make control-plane calls slow (fault injection).
#include <getopt.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <iostream>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "grpc_client.h"
#include "http_client.h"
#include "shm_utils.h"

namespace tc = triton::client;

namespace {

void Fail(const std::string& what, const tc::Error& err)
{
  std::cerr << "error: " << what << ": " << err << std::endl;
  exit(1);
}

#define CHECK_OK(X, MSG)             \
  do {                               \
    tc::Error e__ = (X);             \
    if (!e__.IsOk()) Fail((MSG), e__); \
  } while (false)

// Control plane with a deadline: each failure is reported and counted.
int ControlPlane(tc::InferenceServerGrpcClient* c, uint64_t timeout_ms, const std::string& model,
                 const tc::Headers& h)
{
  int errors = 0;
  auto check = [&](const tc::Error& e, const char* what) {
    if (!e.IsOk()) {
      std::cout << "error: Failed on " << what << ": " << e << std::endl;
      ++errors;
    }
  };
  bool flag = false;
  inference::ServerMetadataResponse smeta;
  inference::ModelMetadataResponse mmeta;
  inference::ModelConfigResponse mcfg;
  inference::RepositoryIndexResponse index;
  inference::ModelStatisticsResponse stats;
  inference::TraceSettingResponse trace;
  inference::SystemSharedMemoryStatusResponse sys_status;
  inference::CudaSharedMemoryStatusResponse dev_status;
  check(c->IsServerLive(&flag, h, timeout_ms), "IsServerLive");
  check(c->IsServerReady(&flag, h, timeout_ms), "IsServerReady");
  check(c->IsModelReady(&flag, model, "", h, timeout_ms), "IsModelReady");
  check(c->ServerMetadata(&smeta, h, timeout_ms), "ServerMetadata");
  check(c->ModelMetadata(&mmeta, model, "", h, timeout_ms), "ModelMetadata");
  check(c->ModelConfig(&mcfg, model, "", h, timeout_ms), "ModelConfig");
  check(c->ModelRepositoryIndex(&index, h, timeout_ms), "ModelRepositoryIndex");
  check(c->ModelInferenceStatistics(&stats, model, "", h, timeout_ms), "ModelInferenceStatistics");
  check(c->LoadModel(model, h, "", {}, timeout_ms), "LoadModel");
  check(c->UnloadModel(model, h, timeout_ms), "UnloadModel");
  check(c->LoadModel(model, h, "", {}, timeout_ms), "LoadModel (reload)");
  check(c->UpdateTraceSettings(&trace, model, {}, h, timeout_ms), "UpdateTraceSettings");
  check(c->GetTraceSettings(&trace, model, h, timeout_ms), "GetTraceSettings");
  // a real system shm region, so register/status/unregister are valid requests
  const std::string key = "/client_timeout_test_" + std::to_string(getpid());
  int fd = -1;
  void* addr = nullptr;
  CHECK_OK(tc::CreateSharedMemoryRegion(key, 64, &fd), "create shm region");
  CHECK_OK(tc::MapSharedMemory(fd, 0, 64, &addr), "map shm region");
  check(c->RegisterSystemSharedMemory("timeout_test_region", key, 64, 0, h, timeout_ms), "RegisterSystemSharedMemory");
  check(c->SystemSharedMemoryStatus(&sys_status, "", h, timeout_ms), "SystemSharedMemoryStatus");
  check(c->UnregisterSystemSharedMemory("timeout_test_region", h, timeout_ms), "UnregisterSystemSharedMemory");
  tc::UnmapSharedMemory(addr, 64);
  tc::CloseSharedMemory(fd);
  tc::UnlinkSharedMemoryRegion(key);
  check(c->CudaSharedMemoryStatus(&dev_status, "", h, timeout_ms), "CudaSharedMemoryStatus");
  check(c->UnregisterCudaSharedMemory("", h, timeout_ms), "UnregisterCudaSharedMemory");
  return errors;
}

void Validate(tc::InferResult* raw, const std::vector<int32_t>& in)
{
  std::shared_ptr<tc::InferResult> r(raw);
  CHECK_OK(r->RequestStatus(), "Inference failed");
  std::vector<int64_t> shape;
  std::string dt;
  CHECK_OK(r->Shape("OUTPUT0", &shape), "unable to get shape for 'OUTPUT0'");
  CHECK_OK(r->Datatype("OUTPUT0", &dt), "unable to get datatype for 'OUTPUT0'");
  if (shape != std::vector<int64_t>{1, 16} || dt != "INT32") {
    std::cerr << "error: received incorrect shape/datatype for 'OUTPUT0'" << std::endl;
    exit(1);
  }
  const uint8_t* data = nullptr;
  size_t n = 0;
  CHECK_OK(r->RawData("OUTPUT0", &data, &n), "unable to get result data for 'OUTPUT0'");
  if (n != 64 || !std::equal(in.begin(), in.end(), reinterpret_cast<const int32_t*>(data))) {
    std::cerr << "error: incorrect output" << std::endl;
    exit(1);
  }
  std::cout << r->DebugString() << std::endl;
}

template <typename Client>
void Sync(Client* c, tc::InferOptions& o, std::vector<tc::InferInput*>& in,
          std::vector<const tc::InferRequestedOutput*>& out, const std::vector<int32_t>& data)
{
  tc::InferResult* r = nullptr;
  CHECK_OK(c->Infer(&r, o, in, out), "unable to run model");
  Validate(r, data);
}

template <typename Client>
void Async(Client* c, tc::InferOptions& o, std::vector<tc::InferInput*>& in,
           std::vector<const tc::InferRequestedOutput*>& out, const std::vector<int32_t>& data)
{
  std::mutex mu;
  std::condition_variable cv;
  tc::InferResult* got = nullptr;
  CHECK_OK(c->AsyncInfer(
               [&](tc::InferResult* r) {
                 std::lock_guard<std::mutex> lk(mu);
                 std::cout << "Callback called" << std::endl;
                 got = r;
                 cv.notify_all();
               },
               o, in, out),
           "unable to run model");
  std::unique_lock<std::mutex> lk(mu);
  cv.wait(lk, [&] { return got != nullptr; });
  Validate(got, data);
}

void Stream(tc::InferenceServerGrpcClient* c, uint32_t timeout_us, tc::InferOptions& o,
            std::vector<tc::InferInput*>& in, const std::vector<int32_t>& data)
{
  std::mutex mu;
  std::condition_variable cv;
  std::vector<tc::InferResult*> got;
  CHECK_OK(c->StartStream(
               [&](tc::InferResult* r) {
                 std::lock_guard<std::mutex> lk(mu);
                 got.push_back(r);
                 cv.notify_all();
               },
               false, timeout_us),
           "Failed to start the stream");
  CHECK_OK(c->AsyncStreamInfer(o, in), "unable to run model");
  {
    std::unique_lock<std::mutex> lk(mu);
    // a stream deadline ends the stream with an error result; without one, wait for the response
    const auto limit = std::chrono::microseconds(timeout_us ? timeout_us : 60000000u) + std::chrono::seconds(5);
    if (!cv.wait_for(lk, limit, [&] { return !got.empty(); })) {
      std::cerr << "Stream has been closed" << std::endl;
      exit(1);
    }
  }
  if (got.size() != 1) {
    std::cerr << "error: expected a single response, got " << got.size() << std::endl;
    exit(1);
  }
  Validate(got[0], data);
  c->StopStream();
}

void Usage(char** argv)
{
  std::cerr << "Usage: " << argv[0] << " [options]\n"
            << "\t-v\n\t-i <http|grpc>\n\t-u <URL for inference service>\n"
            << "\t-a (async)\n\t-s (gRPC streaming)\n\t-t <client timeout in microseconds>\n"
            << "\t-p (gRPC: control-plane APIs with timeout_ms = -t)\n\t-H <header:value>\n";
  exit(1);
}

}  // namespace

int main(int argc, char** argv)
{
  bool verbose = false, async = false, streaming = false, apis = false;
  std::string protocol = "http", url;
  uint32_t timeout = 0;
  tc::Headers headers;
  int opt;
  while ((opt = getopt(argc, argv, "vi:u:ast:pH:")) != -1) {
    switch (opt) {
      case 'v': verbose = true; break;
      case 'i': {
        std::string p(optarg);
        std::transform(p.begin(), p.end(), p.begin(), ::tolower);
        protocol = (p == "grpc" || p == "http") ? p : "unknown";
        break;
      }
      case 'u': url = optarg; break;
      case 'a': async = true; break;
      case 's': streaming = true; break;
      case 't': timeout = static_cast<uint32_t>(std::stoul(optarg)); break;
      case 'p': apis = true; break;
      case 'H': {
        std::string kv(optarg);
        const size_t c = kv.find(':');
        if (c == std::string::npos) Usage(argv);
        headers[kv.substr(0, c)] = kv.substr(c + 1);
        break;
      }
      default: Usage(argv);
    }
  }
  if (protocol == "unknown" || (streaming && protocol != "grpc")) {
    std::cerr << "Supports only http and grpc protocols (streaming: grpc)" << std::endl;
    Usage(argv);
  }
  const std::string model = "custom_identity_int32";
  std::unique_ptr<tc::InferenceServerGrpcClient> grpc;
  std::unique_ptr<tc::InferenceServerHttpClient> http;
  if (protocol == "grpc") {
    CHECK_OK(tc::InferenceServerGrpcClient::Create(&grpc, url.empty() ? "localhost:8001" : url, verbose),
             "unable to create grpc client");
  } else {
    CHECK_OK(tc::InferenceServerHttpClient::Create(&http, url.empty() ? "localhost:8000" : url, verbose),
             "unable to create http client");
  }
  if (apis) {
    if (!grpc) Usage(argv);
    const int errors = ControlPlane(grpc.get(), timeout, model, headers);
    if (errors) {
      std::cerr << "error count: " << errors << " which is not 0" << std::endl;
      return 1;
    }
    std::cout << "PASS: control-plane APIs" << std::endl;
    return 0;
  }
  std::vector<int32_t> data(16);
  for (int i = 0; i < 16; ++i) data[i] = i;
  tc::InferInput* in0 = nullptr;
  CHECK_OK(tc::InferInput::Create(&in0, "INPUT0", {1, 16}, "INT32"), "unable to get INPUT0");
  std::unique_ptr<tc::InferInput> in0p(in0);
  CHECK_OK(in0->AppendRaw(reinterpret_cast<const uint8_t*>(data.data()), 64), "unable to set data for INPUT0");
  tc::InferRequestedOutput* out0 = nullptr;
  CHECK_OK(tc::InferRequestedOutput::Create(&out0, "OUTPUT0"), "unable to get 'OUTPUT0'");
  std::unique_ptr<tc::InferRequestedOutput> out0p(out0);
  std::vector<tc::InferInput*> inputs{in0};
  std::vector<const tc::InferRequestedOutput*> outputs{out0};
  tc::InferOptions options(model);
  options.client_timeout_ = timeout;
  if (streaming) {
    Stream(grpc.get(), timeout, options, inputs, data);
  } else if (grpc) {
    async ? Async(grpc.get(), options, inputs, outputs, data) : Sync(grpc.get(), options, inputs, outputs, data);
  } else {
    async ? Async(http.get(), options, inputs, outputs, data) : Sync(http.get(), options, inputs, outputs, data);
  }
  std::cout << "PASS: infer" << std::endl;
  return 0;
}

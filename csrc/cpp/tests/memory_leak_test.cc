// memory_leak_test: soak the C++ clients with repeated sync inference on
// `custom_identity_int32`, either re-creating the client every repetition
// (default) or reusing one (-R) — behavioral parity with reference
// src/c++/tests/memory_leak_test.cc (same CLI, same retry-on-error policy).
// The reference relies on an external leak checker; this port also measures
// its own resident set size and fails when it grows by more than -m KiB
// between the end of the warm-up repetitions and the last repetition.
//
//   memory_leak_test [-v] [-i http|grpc] [-u url] [-r reps] [-R] [-m max_growth_kib] [-w retry_sleep_s]
//                    [-M model (INT32 [1,16] identity; default custom_identity_int32)]
#include <getopt.h>
#include <unistd.h>

#include <algorithm>
#include <fstream>
#include <iostream>
#include <memory>
#include <string>
#include <vector>

#include "grpc_client.h"
#include "http_client.h"

namespace tc = triton::client;

namespace {

constexpr int kDim = 16;

long RssKiB()
{
  std::ifstream f("/proc/self/status");
  std::string line;
  while (std::getline(f, line))
    if (line.rfind("VmRSS:", 0) == 0) return std::stol(line.substr(6));
  return -1;
}

void Fail(const std::string& what, const tc::Error& e)
{
  std::cerr << "error: " << what << ": " << e << std::endl;
  exit(1);
}

template <typename Client>
void InferWithRetries(Client* c, tc::InferResult** r, tc::InferOptions& o, std::vector<tc::InferInput*>& in,
                      std::vector<const tc::InferRequestedOutput*>& out, int retry_sleep_s)
{
  // socket exhaustion under many short-lived clients is retried, not fatal
  constexpr int kMaxRetries = 5;
  tc::Error err = c->Infer(r, o, in, out);
  for (int i = 0; !err.IsOk() && i < kMaxRetries; ++i) {
    std::cerr << "Error: " << err << "\nSleeping for " << retry_sleep_s << " seconds and retrying. [Attempt: "
              << i + 1 << "/" << kMaxRetries << "]" << std::endl;
    sleep(retry_sleep_s);
    err = c->Infer(r, o, in, out);
  }
  if (!err.IsOk()) {
    std::cerr << "error: Exceeded max tries [" << kMaxRetries << "] on inference without success" << std::endl;
    exit(1);
  }
}

void Validate(tc::InferResult* raw, const std::vector<int32_t>& in)
{
  std::unique_ptr<tc::InferResult> r(raw);
  if (!r->RequestStatus().IsOk()) Fail("Inference failed", r->RequestStatus());
  const uint8_t* d = nullptr;
  size_t n = 0;
  tc::Error e = r->RawData("OUTPUT0", &d, &n);
  if (!e.IsOk()) Fail("unable to get result data for 'OUTPUT0'", e);
  if (n != kDim * sizeof(int32_t) || !std::equal(in.begin(), in.end(), reinterpret_cast<const int32_t*>(d))) {
    std::cerr << "error: incorrect output" << std::endl;
    exit(1);
  }
}

template <typename Client>
long Run(const std::string& url, const std::string& model, bool verbose, bool reuse, uint32_t reps,
         int retry_sleep_s, long* rss_warm)
{
  std::vector<int32_t> data(kDim);
  for (int i = 0; i < kDim; ++i) data[i] = i;
  tc::InferInput* in0 = nullptr;
  tc::Error e = tc::InferInput::Create(&in0, "INPUT0", {1, kDim}, "INT32");
  if (!e.IsOk()) Fail("unable to get INPUT0", e);
  std::unique_ptr<tc::InferInput> in0p(in0);
  e = in0->AppendRaw(reinterpret_cast<const uint8_t*>(data.data()), data.size() * sizeof(int32_t));
  if (!e.IsOk()) Fail("unable to set data for INPUT0", e);
  tc::InferRequestedOutput* out0 = nullptr;
  e = tc::InferRequestedOutput::Create(&out0, "OUTPUT0");
  if (!e.IsOk()) Fail("unable to get 'OUTPUT0'", e);
  std::unique_ptr<tc::InferRequestedOutput> out0p(out0);
  std::vector<tc::InferInput*> inputs{in0};
  std::vector<const tc::InferRequestedOutput*> outputs{out0};
  tc::InferOptions options(model);

  const uint32_t warm = std::max<uint32_t>(1, reps / 10);
  std::unique_ptr<Client> client;
  e = Client::Create(&client, url, verbose);
  if (!e.IsOk()) Fail("unable to create client", e);
  for (uint32_t i = 0; i < reps; ++i) {
    if (!reuse) {
      e = Client::Create(&client, url, verbose);
      if (!e.IsOk()) Fail("unable to create client", e);
    }
    tc::InferResult* r = nullptr;
    InferWithRetries(client.get(), &r, options, inputs, outputs, retry_sleep_s);
    Validate(r, data);
    if (i + 1 == warm) *rss_warm = RssKiB();
  }
  client.reset();
  return RssKiB();
}

void Usage(char** argv)
{
  std::cerr << "Usage: " << argv[0] << " [options]\n"
            << "\t-v\n\t-i <http/grpc>\n\t-u <URL for inference service>\n"
            << "\t-r <number of repetitions for inference> default is 100.\n"
            << "\t-R Re-use the same client for each repetition. Without this flag, the default is to create a new "
               "client on each repetition.\n"
            << "\t-m <max RSS growth in KiB after warm-up> default 8192 (0 = report only)\n"
            << "\t-w <seconds to sleep before a retry> default 60\n"
            << "\t-M <model name> default custom_identity_int32\n";
  exit(1);
}

}  // namespace

int main(int argc, char** argv)
{
  bool verbose = false, reuse = false;
  std::string protocol = "http", url, model = "custom_identity_int32";
  uint32_t reps = 100;
  long max_growth = 8192;
  int retry_sleep_s = 60;
  int opt;
  while ((opt = getopt(argc, argv, "vi:u:r:Rm:w:M:")) != -1) {
    switch (opt) {
      case 'v': verbose = true; break;
      case 'i': {
        std::string p(optarg);
        std::transform(p.begin(), p.end(), p.begin(), ::tolower);
        protocol = (p == "grpc" || p == "http") ? p : "unknown";
        break;
      }
      case 'u': url = optarg; break;
      case 'r': reps = static_cast<uint32_t>(std::stoul(optarg)); break;
      case 'R': reuse = true; break;
      case 'm': max_growth = std::stol(optarg); break;
      case 'w': retry_sleep_s = std::stoi(optarg); break;
      case 'M': model = optarg; break;
      default: Usage(argv);
    }
  }
  if (protocol == "unknown") {
    std::cerr << "Supports only http and grpc protocols" << std::endl;
    Usage(argv);
  }
  long warm = -1, end = -1;
  if (protocol == "grpc")
    end = Run<tc::InferenceServerGrpcClient>(url.empty() ? "localhost:8001" : url, model, verbose, reuse, reps,
                                             retry_sleep_s, &warm);
  else
    end = Run<tc::InferenceServerHttpClient>(url.empty() ? "localhost:8000" : url, model, verbose, reuse, reps,
                                             retry_sleep_s, &warm);
  const long growth = end - warm;
  std::cout << "repetitions " << reps << (reuse ? " (reused client)" : " (new client each)") << ": RSS after warm-up "
            << warm << " KiB, at end " << end << " KiB, growth " << growth << " KiB" << std::endl;
  if (max_growth > 0 && growth > max_growth) {
    std::cerr << "error: RSS grew by " << growth << " KiB (limit " << max_growth << ")" << std::endl;
    return 1;
  }
  std::cout << "PASS" << std::endl;
  return 0;
}

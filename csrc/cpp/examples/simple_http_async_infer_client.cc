// Async HTTP inference: several requests in flight, completions delivered to
// a callback (reference src/c++/examples/simple_http_async_infer_client.cc).
#include <getopt.h>

#include <condition_variable>
#include <mutex>

#include "example_util.h"
#include "http_client.h"

namespace tc = triton::client;

int main(int argc, char** argv)
{
  bool verbose = false;
  std::string url("localhost:8000");
  tc::Headers headers;
  int opt;
  while ((opt = getopt(argc, argv, "vu:H:")) != -1) {
    switch (opt) {
      case 'v': verbose = true; break;
      case 'u': url = optarg; break;
      case 'H': example::AddHeader(&headers, optarg); break;
      default: example::Usage(argv);
    }
  }
  std::unique_ptr<tc::InferenceServerHttpClient> client;
  FAIL_IF_ERR(tc::InferenceServerHttpClient::Create(&client, url, verbose), "unable to create client");
  example::SimpleData d;
  tc::InferInput *in0, *in1;
  FAIL_IF_ERR(tc::InferInput::Create(&in0, "INPUT0", {1, 16}, "INT32"), "unable to get INPUT0");
  FAIL_IF_ERR(tc::InferInput::Create(&in1, "INPUT1", {1, 16}, "INT32"), "unable to get INPUT1");
  std::unique_ptr<tc::InferInput> p0(in0), p1(in1);
  FAIL_IF_ERR(in0->AppendRaw(reinterpret_cast<uint8_t*>(d.in0.data()), 64), "unable to set data for INPUT0");
  FAIL_IF_ERR(in1->AppendRaw(reinterpret_cast<uint8_t*>(d.in1.data()), 64), "unable to set data for INPUT1");
  tc::InferRequestedOutput *o0, *o1;
  FAIL_IF_ERR(tc::InferRequestedOutput::Create(&o0, "OUTPUT0"), "unable to get OUTPUT0");
  FAIL_IF_ERR(tc::InferRequestedOutput::Create(&o1, "OUTPUT1"), "unable to get OUTPUT1");
  std::unique_ptr<tc::InferRequestedOutput> q0(o0), q1(o1);
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::unique_ptr<tc::InferResult>> results;
  const int n = 4;
  for (int i = 0; i < n; ++i) {
    tc::InferOptions options("simple");
    options.request_id_ = std::to_string(i);
    FAIL_IF_ERR(client->AsyncInfer(
                    [&](tc::InferResult* r) {
                      std::lock_guard<std::mutex> lk(mu);
                      results.emplace_back(r);
                      cv.notify_all();
                    },
                    options, {in0, in1}, {o0, o1}, headers),
                "unable to run model");
  }
  {
    std::unique_lock<std::mutex> lk(mu);
    if (!cv.wait_for(lk, std::chrono::seconds(60), [&] { return (int)results.size() == n; })) {
      std::cerr << "error: timed out waiting for the results" << std::endl;
      exit(1);
    }
  }
  for (auto& r : results) {
    FAIL_IF_ERR(r->RequestStatus(), "inference failed");
    example::ValidateSimple(r.get(), d, false);
  }
  std::cout << "PASS : Async Infer" << std::endl;
  return 0;
}

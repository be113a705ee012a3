// Decoupled model `repeat_int32` over a gRPC stream: one request, one
// response per element (reference src/c++/examples/simple_grpc_custom_repeat.cc).
#include <getopt.h>

#include <condition_variable>
#include <mutex>

#include "example_util.h"
#include "grpc_client.h"

namespace tc = triton::client;

int main(int argc, char** argv)
{
  bool verbose = false;
  std::string url("localhost:8001");
  int repeat = 4;
  int opt;
  while ((opt = getopt(argc, argv, "vu:r:")) != -1) {
    switch (opt) {
      case 'v': verbose = true; break;
      case 'u': url = optarg; break;
      case 'r': repeat = std::stoi(optarg); break;
      default: example::Usage(argv, "\t-r <number of responses>");
    }
  }
  std::unique_ptr<tc::InferenceServerGrpcClient> client;
  FAIL_IF_ERR(tc::InferenceServerGrpcClient::Create(&client, url, verbose), "unable to create grpc client");
  std::mutex mu;
  std::condition_variable cv;
  std::vector<int32_t> got;
  bool failed = false;
  FAIL_IF_ERR(client->StartStream([&](tc::InferResult* r) {
    std::unique_ptr<tc::InferResult> rr(r);
    std::lock_guard<std::mutex> lk(mu);
    const uint8_t* buf;
    size_t n;
    bool null_resp = false;
    r->IsNullResponse(&null_resp);
    if (!r->RequestStatus().IsOk()) failed = true;
    else if (!null_resp && r->RawData("OUT", &buf, &n).IsOk()) got.push_back(*reinterpret_cast<const int32_t*>(buf));
    cv.notify_all();
  }),
              "unable to start stream");
  std::vector<int32_t> values(repeat);
  std::vector<uint32_t> delays(repeat, 0);
  uint32_t wait = 0;
  for (int i = 0; i < repeat; ++i) values[i] = i * 10;
  tc::InferInput *in, *delay, *w;
  FAIL_IF_ERR(tc::InferInput::Create(&in, "IN", {repeat}, "INT32"), "IN");
  FAIL_IF_ERR(tc::InferInput::Create(&delay, "DELAY", {repeat}, "UINT32"), "DELAY");
  FAIL_IF_ERR(tc::InferInput::Create(&w, "WAIT", {1}, "UINT32"), "WAIT");
  std::unique_ptr<tc::InferInput> p0(in), p1(delay), p2(w);
  in->AppendRaw(reinterpret_cast<uint8_t*>(values.data()), values.size() * 4);
  delay->AppendRaw(reinterpret_cast<uint8_t*>(delays.data()), delays.size() * 4);
  w->AppendRaw(reinterpret_cast<uint8_t*>(&wait), 4);
  tc::InferOptions options("repeat_int32");
  FAIL_IF_ERR(client->AsyncStreamInfer(options, {in, delay, w}), "unable to send request");
  {
    std::unique_lock<std::mutex> lk(mu);
    if (!cv.wait_for(lk, std::chrono::seconds(60), [&] { return failed || (int)got.size() == repeat; })) {
      std::cerr << "error: got " << got.size() << " of " << repeat << " responses" << std::endl;
      exit(1);
    }
  }
  client->StopStream();
  if (failed) {
    std::cerr << "error: a response reported an error" << std::endl;
    exit(1);
  }
  for (int i = 0; i < repeat; ++i) {
    std::cout << "response " << i << ": " << got[i] << std::endl;
    if (got[i] != values[i]) {
      std::cerr << "error: unexpected response order/value" << std::endl;
      exit(1);
    }
  }
  std::cout << "PASS : Custom Repeat" << std::endl;
  return 0;
}

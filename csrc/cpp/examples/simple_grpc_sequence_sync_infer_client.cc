// Two interleaved stateful sequences over GRPC on `simple_sequence`
// (-d: `simple_dyna_sequence`) (reference src/c++/examples/simple_grpc_sequence_sync_infer_client.cc).
#include <getopt.h>

#include "example_util.h"
#include "grpc_client.h"

namespace tc = triton::client;

static int32_t Step(tc::InferenceServerGrpcClient* client, const std::string& model, int32_t value, uint64_t seq, bool start, bool end)
{
  tc::InferInput* in;
  FAIL_IF_ERR(tc::InferInput::Create(&in, "INPUT", {1, 1}, "INT32"), "unable to create INPUT");
  std::unique_ptr<tc::InferInput> p(in);
  FAIL_IF_ERR(in->AppendRaw(reinterpret_cast<uint8_t*>(&value), 4), "unable to set INPUT");
  tc::InferOptions options(model);
  options.sequence_id_ = seq;
  options.sequence_start_ = start;
  options.sequence_end_ = end;
  tc::InferResult* result;
  FAIL_IF_ERR(client->Infer(&result, options, {in}), "unable to run model");
  std::unique_ptr<tc::InferResult> r(result);
  FAIL_IF_ERR(result->RequestStatus(), "inference failed");
  const uint8_t* buf;
  size_t n;
  FAIL_IF_ERR(result->RawData("OUTPUT", &buf, &n), "unable to get OUTPUT");
  return *reinterpret_cast<const int32_t*>(buf);
}

int main(int argc, char** argv)
{
  bool verbose = false, dyna = false;
  std::string url("localhost:8001");
  int opt;
  while ((opt = getopt(argc, argv, "vdu:")) != -1) {
    switch (opt) {
      case 'v': verbose = true; break;
      case 'd': dyna = true; break;
      case 'u': url = optarg; break;
      default: example::Usage(argv, "\t-d use simple_dyna_sequence");
    }
  }
  const std::string model = dyna ? "simple_dyna_sequence" : "simple_sequence";
  std::unique_ptr<tc::InferenceServerGrpcClient> client;
  FAIL_IF_ERR(tc::InferenceServerGrpcClient::Create(&client, url, verbose), "unable to create client");
  const std::vector<int32_t> values = {11, 7, 5, 3, 2, 0, 1};
  const uint64_t s0 = 1000, s1 = 1001;
  std::vector<int32_t> r0, r1;
  r0.push_back(Step(client.get(), model, 0, s0, true, false));
  r1.push_back(Step(client.get(), model, 100, s1, true, false));
  for (size_t i = 0; i < values.size(); ++i) {
    const bool end = i + 1 == values.size();
    r0.push_back(Step(client.get(), model, values[i], s0, false, end));
    r1.push_back(Step(client.get(), model, -values[i], s1, false, end));
  }
  for (size_t i = 0; i < r0.size(); ++i) std::cout << "[" << i << "] " << r0[i] << " : " << r1[i] << std::endl;
  if (r0 == r1) {
    std::cerr << "error: the two sequences interfered" << std::endl;
    exit(1);
  }
  std::cout << "PASS : Sequence" << std::endl;
  return 0;
}

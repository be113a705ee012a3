// BYTES tensors on `simple_string` over GRPC (reference
// src/c++/examples/simple_grpc_string_infer_client.cc).
#include <getopt.h>

#include "example_util.h"
#include "grpc_client.h"

namespace tc = triton::client;

int main(int argc, char** argv)
{
  bool verbose = false;
  std::string url("localhost:8001");
  int opt;
  while ((opt = getopt(argc, argv, "vu:")) != -1) {
    switch (opt) {
      case 'v': verbose = true; break;
      case 'u': url = optarg; break;
      default: example::Usage(argv);
    }
  }
  std::unique_ptr<tc::InferenceServerGrpcClient> client;
  FAIL_IF_ERR(tc::InferenceServerGrpcClient::Create(&client, url, verbose), "unable to create client");
  std::vector<std::string> a, b;
  for (int i = 0; i < 16; ++i) {
    a.push_back(std::to_string(i));
    b.push_back("1");
  }
  tc::InferInput *in0, *in1;
  FAIL_IF_ERR(tc::InferInput::Create(&in0, "INPUT0", {1, 16}, "BYTES"), "unable to get INPUT0");
  FAIL_IF_ERR(tc::InferInput::Create(&in1, "INPUT1", {1, 16}, "BYTES"), "unable to get INPUT1");
  std::unique_ptr<tc::InferInput> p0(in0), p1(in1);
  FAIL_IF_ERR(in0->AppendFromString(a), "unable to set data for INPUT0");
  FAIL_IF_ERR(in1->AppendFromString(b), "unable to set data for INPUT1");
  tc::InferRequestedOutput *o0, *o1;
  FAIL_IF_ERR(tc::InferRequestedOutput::Create(&o0, "OUTPUT0"), "unable to get OUTPUT0");
  FAIL_IF_ERR(tc::InferRequestedOutput::Create(&o1, "OUTPUT1"), "unable to get OUTPUT1");
  std::unique_ptr<tc::InferRequestedOutput> q0(o0), q1(o1);
  tc::InferOptions options("simple_string");
  tc::InferResult* result;
  FAIL_IF_ERR(client->Infer(&result, options, {in0, in1}, {o0, o1}), "unable to run model");
  std::unique_ptr<tc::InferResult> r(result);
  FAIL_IF_ERR(result->RequestStatus(), "inference failed");
  std::vector<std::string> s, dd;
  FAIL_IF_ERR(result->StringData("OUTPUT0", &s), "unable to get OUTPUT0");
  FAIL_IF_ERR(result->StringData("OUTPUT1", &dd), "unable to get OUTPUT1");
  for (int i = 0; i < 16; ++i) {
    std::cout << a[i] << " + " << b[i] << " = " << s[i] << std::endl;
    std::cout << a[i] << " - " << b[i] << " = " << dd[i] << std::endl;
    if (std::stoi(s[i]) != i + 1 || std::stoi(dd[i]) != i - 1) {
      std::cerr << "error: incorrect result" << std::endl;
      exit(1);
    }
  }
  std::cout << "PASS : String Infer" << std::endl;
  return 0;
}

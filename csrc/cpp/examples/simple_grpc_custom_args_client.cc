// gRPC client with explicit grpc::ChannelArguments (reference
// src/c++/examples/simple_grpc_custom_args_client.cc).
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
  grpc::ChannelArguments args;
  args.SetMaxSendMessageSize(tc::MAX_GRPC_MESSAGE_SIZE);
  args.SetMaxReceiveMessageSize(tc::MAX_GRPC_MESSAGE_SIZE);
  args.SetString("grpc.lb_policy_name", "pick_first");
  args.SetInt("grpc.keepalive_time_ms", INT32_MAX);
  FAIL_IF_ERR(tc::InferenceServerGrpcClient::Create(&client, url, args, verbose), "unable to create grpc client");
  example::SimpleData d;
  tc::InferInput *in0, *in1;
  FAIL_IF_ERR(tc::InferInput::Create(&in0, "INPUT0", {1, 16}, "INT32"), "unable to get INPUT0");
  FAIL_IF_ERR(tc::InferInput::Create(&in1, "INPUT1", {1, 16}, "INT32"), "unable to get INPUT1");
  std::unique_ptr<tc::InferInput> p0(in0), p1(in1);
  FAIL_IF_ERR(in0->AppendRaw(reinterpret_cast<uint8_t*>(d.in0.data()), 64), "unable to set data for INPUT0");
  FAIL_IF_ERR(in1->AppendRaw(reinterpret_cast<uint8_t*>(d.in1.data()), 64), "unable to set data for INPUT1");
  tc::InferOptions options("simple");
  tc::InferResult* result;
  FAIL_IF_ERR(client->Infer(&result, options, {in0, in1}), "unable to run model");
  std::unique_ptr<tc::InferResult> r(result);
  FAIL_IF_ERR(result->RequestStatus(), "inference failed");
  example::ValidateSimple(result, d);
  std::cout << "PASS : Infer" << std::endl;
  return 0;
}

// Model repository control over GRPC: index, unload, load, load with a config
// override (reference src/c++/examples/simple_grpc_model_control.cc).
#include <getopt.h>

#include "example_util.h"
#include "grpc_client.h"

namespace tc = triton::client;

static void ExpectReady(tc::InferenceServerGrpcClient* client, bool want)
{
  bool ready = !want;
  FAIL_IF_ERR(client->IsModelReady(&ready, "simple"), "unable to get model readiness");
  if (ready != want) {
    std::cerr << "error: expected model 'simple' to be " << (want ? "ready" : "unavailable") << std::endl;
    exit(1);
  }
}

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
  inference::RepositoryIndexResponse idx; FAIL_IF_ERR(client->ModelRepositoryIndex(&idx), "unable to get repository index"); std::cout << idx.DebugString() << std::endl;
  FAIL_IF_ERR(client->UnloadModel("simple"), "unable to unload model");
  ExpectReady(client.get(), false);
  FAIL_IF_ERR(client->LoadModel("simple"), "unable to load model");
  ExpectReady(client.get(), true);
  tc::Error e = client->LoadModel("wrong_model_name");
  if (e.IsOk()) {
    std::cerr << "error: expected failure loading a wrong model name" << std::endl;
    exit(1);
  }
  std::cout << "expected error: " << e << std::endl;
  FAIL_IF_ERR(client->LoadModel("simple", tc::Headers(), "{\"max_batch_size\":8,\"version_policy\":{\"latest\":{\"num_versions\":1}}}"), "unable to load model with config override");
  ExpectReady(client.get(), true);
  std::cout << "PASS : Model Control" << std::endl;
  return 0;
}

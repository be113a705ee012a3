// Health, server/model metadata, config and statistics over gRPC (reference
// src/c++/examples/simple_grpc_health_metadata.cc).
#include <getopt.h>

#include "example_util.h"
#include "grpc_client.h"

namespace tc = triton::client;

int main(int argc, char** argv)
{
  bool verbose = false;
  std::string url("localhost:8001");
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
  std::unique_ptr<tc::InferenceServerGrpcClient> client;
  FAIL_IF_ERR(tc::InferenceServerGrpcClient::Create(&client, url, verbose), "unable to create grpc client");
  bool live, ready, model_ready;
  FAIL_IF_ERR(client->IsServerLive(&live, headers), "unable to get server liveness");
  FAIL_IF_ERR(client->IsServerReady(&ready, headers), "unable to get server readiness");
  FAIL_IF_ERR(client->IsModelReady(&model_ready, "simple", "", headers), "unable to get model readiness");
  if (!live || !ready || !model_ready) {
    std::cerr << "error: server or model not ready" << std::endl;
    exit(1);
  }
  inference::ServerMetadataResponse md;
  FAIL_IF_ERR(client->ServerMetadata(&md, headers), "unable to get server metadata");
  std::cout << md.DebugString() << std::endl;
  inference::ModelMetadataResponse mm;
  FAIL_IF_ERR(client->ModelMetadata(&mm, "simple", "", headers), "unable to get model metadata");
  if (mm.name() != "simple" || mm.inputs_size() != 2) {
    std::cerr << "error: unexpected model metadata" << std::endl;
    exit(1);
  }
  std::cout << mm.DebugString() << std::endl;
  inference::ModelConfigResponse cfg;
  FAIL_IF_ERR(client->ModelConfig(&cfg, "simple", "", headers), "unable to get model config");
  if (cfg.config().name() != "simple") {
    std::cerr << "error: unexpected model config" << std::endl;
    exit(1);
  }
  std::cout << cfg.DebugString() << std::endl;
  inference::ModelStatisticsResponse st;
  FAIL_IF_ERR(client->ModelInferenceStatistics(&st, "simple", "", headers), "unable to get statistics");
  std::cout << st.DebugString() << std::endl;
  inference::ModelMetadataResponse bad;
  tc::Error e = client->ModelMetadata(&bad, "wrong_model_name", "", headers);
  if (e.IsOk()) {
    std::cerr << "error: expected an error for a wrong model name" << std::endl;
    exit(1);
  }
  std::cout << "expected error: " << e << std::endl;
  std::cout << "PASS : Health Metadata" << std::endl;
  return 0;
}

// Health, server/model metadata, config and statistics over HTTP (reference
// src/c++/examples/simple_http_health_metadata.cc).
#include <getopt.h>

#include "example_util.h"
#include "http_client.h"
#include "json.h"

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
  FAIL_IF_ERR(tc::InferenceServerHttpClient::Create(&client, url, verbose), "unable to create http client");
  bool live, ready, model_ready;
  FAIL_IF_ERR(client->IsServerLive(&live, headers), "unable to get server liveness");
  FAIL_IF_ERR(client->IsServerReady(&ready, headers), "unable to get server readiness");
  FAIL_IF_ERR(client->IsModelReady(&model_ready, "simple", "", headers), "unable to get model readiness");
  if (!live || !ready || !model_ready) {
    std::cerr << "error: server or model not ready" << std::endl;
    exit(1);
  }
  std::string md, mm, cfg, st;
  FAIL_IF_ERR(client->ServerMetadata(&md, headers), "unable to get server metadata");
  FAIL_IF_ERR(client->ModelMetadata(&mm, "simple", "", headers), "unable to get model metadata");
  FAIL_IF_ERR(client->ModelConfig(&cfg, "simple", "", headers), "unable to get model config");
  FAIL_IF_ERR(client->ModelInferenceStatistics(&st, "simple", "", headers), "unable to get statistics");
  std::cout << md << std::endl << mm << std::endl << cfg << std::endl << st << std::endl;
  tc::json::Value v;
  std::string err;
  if (!tc::json::Parse(mm, &v, &err) || !v.Find("name") || v.Find("name")->AsString() != "simple") {
    std::cerr << "error: unexpected model metadata" << std::endl;
    exit(1);
  }
  std::string unused;
  tc::Error e = client->ModelMetadata(&unused, "wrong_model_name", "", headers);
  if (e.IsOk()) {
    std::cerr << "error: expected an error for a wrong model name" << std::endl;
    exit(1);
  }
  std::cout << "expected error: " << e << std::endl;
  std::cout << "PASS : Health Metadata" << std::endl;
  return 0;
}

// Raw image file bytes as a BYTES tensor through `preprocess_inception_ensemble`
// (server-side decode + preprocessing + classification) (reference
// src/c++/examples/ensemble_image_client.cc).
#include <getopt.h>

#include <fstream>
#include <sstream>

#include "example_util.h"
#include "grpc_client.h"
#include "http_client.h"

namespace tc = triton::client;

int main(int argc, char** argv)
{
  bool verbose = false;
  int topk = 1;
  std::string url, protocol = "http", model = "preprocess_inception_ensemble";
  int opt;
  while ((opt = getopt(argc, argv, "vc:u:i:m:")) != -1) {
    switch (opt) {
      case 'v': verbose = true; break;
      case 'c': topk = std::stoi(optarg); break;
      case 'u': url = optarg; break;
      case 'i': protocol = optarg; break;
      case 'm': model = optarg; break;
      default: example::Usage(argv, "\t-c <classes> -i <http|grpc> <image file>");
    }
  }
  if (optind >= argc) example::Usage(argv, "\tan image file is required");
  for (auto& ch : protocol) ch = static_cast<char>(tolower(ch));
  std::ifstream f(argv[optind], std::ios::binary);
  if (!f) {
    std::cerr << "error: cannot read " << argv[optind] << std::endl;
    exit(1);
  }
  std::stringstream ss;
  ss << f.rdbuf();
  tc::InferInput* in;
  FAIL_IF_ERR(tc::InferInput::Create(&in, "INPUT", {1, 1}, "BYTES"), "unable to create INPUT");
  std::unique_ptr<tc::InferInput> pin(in);
  FAIL_IF_ERR(in->AppendFromString({ss.str()}), "unable to set INPUT");
  tc::InferRequestedOutput* out;
  FAIL_IF_ERR(tc::InferRequestedOutput::Create(&out, "OUTPUT", topk), "unable to create OUTPUT");
  std::unique_ptr<tc::InferRequestedOutput> pout(out);
  tc::InferOptions options(model);
  tc::InferResult* result;
  if (protocol == "grpc") {
    std::unique_ptr<tc::InferenceServerGrpcClient> c;
    FAIL_IF_ERR(tc::InferenceServerGrpcClient::Create(&c, url.empty() ? "localhost:8001" : url, verbose), "client");
    FAIL_IF_ERR(c->Infer(&result, options, {in}, {out}), "unable to run model");
  } else {
    std::unique_ptr<tc::InferenceServerHttpClient> c;
    FAIL_IF_ERR(tc::InferenceServerHttpClient::Create(&c, url.empty() ? "localhost:8000" : url, verbose), "client");
    FAIL_IF_ERR(c->Infer(&result, options, {in}, {out}), "unable to run model");
  }
  std::unique_ptr<tc::InferResult> r(result);
  FAIL_IF_ERR(result->RequestStatus(), "inference failed");
  std::vector<std::string> classes;
  FAIL_IF_ERR(result->StringData("OUTPUT", &classes), "unable to get OUTPUT");
  if (classes.size() != static_cast<size_t>(topk)) {
    std::cerr << "error: expected " << topk << " classes, got " << classes.size() << std::endl;
    exit(1);
  }
  std::cout << "Image '" << argv[optind] << "':" << std::endl;
  for (const auto& c : classes) std::cout << "    " << c << std::endl;
  std::cout << "PASS" << std::endl;
  return 0;
}

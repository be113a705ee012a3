// Sync gRPC inference on `simple`, with optional compression and client
// timeout (reference src/c++/examples/simple_grpc_infer_client.cc).
#include <getopt.h>

#include "example_util.h"
#include "grpc_client.h"

namespace tc = triton::client;

int main(int argc, char** argv)
{
  bool verbose = false;
  std::string url("localhost:8001");
  tc::Headers headers;
  uint64_t client_timeout = 0;
  grpc_compression_algorithm comp = GRPC_COMPRESS_NONE;
  bool use_ssl = false;
  tc::SslOptions ssl_options;
  // TLS flags of the reference example: --ssl --root-certificates --private-key --certificate-chain
  static const struct option longopts[] = {{"ssl", no_argument, nullptr, 1000},
                                           {"root-certificates", required_argument, nullptr, 1001},
                                           {"private-key", required_argument, nullptr, 1002},
                                           {"certificate-chain", required_argument, nullptr, 1003},
                                           {nullptr, 0, nullptr, 0}};
  int opt;
  while ((opt = getopt_long(argc, argv, "vu:H:t:C:", longopts, nullptr)) != -1) {
    switch (opt) {
      case 1000: use_ssl = true; break;
      case 1001: ssl_options.root_certificates = optarg; break;
      case 1002: ssl_options.private_key = optarg; break;
      case 1003: ssl_options.certificate_chain = optarg; break;
      case 'v': verbose = true; break;
      case 'u': url = optarg; break;
      case 'H': example::AddHeader(&headers, optarg); break;
      case 't': client_timeout = std::stoul(optarg); break;
      case 'C': comp = std::string(optarg) == "gzip" ? GRPC_COMPRESS_GZIP : GRPC_COMPRESS_DEFLATE; break;
      default:
        example::Usage(argv, "\t-t <client timeout in microseconds>\n\t-C <grpc compression: gzip|deflate>\n"
                             "\t--ssl --root-certificates <pem> --private-key <pem> --certificate-chain <pem>");
    }
  }
  std::unique_ptr<tc::InferenceServerGrpcClient> client;
  FAIL_IF_ERR(tc::InferenceServerGrpcClient::Create(&client, url, verbose, use_ssl, ssl_options),
              "unable to create grpc client");
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
  tc::InferOptions options("simple");
  options.client_timeout_ = client_timeout;
  tc::InferResult* result;
  tc::Error e = client->Infer(&result, options, {in0, in1}, {o0, o1}, headers, comp);
  if (!e.IsOk()) {
    if (e.Message().find("Deadline Exceeded") != std::string::npos) {
      std::cerr << "error: Deadline Exceeded" << std::endl;
    }
    std::cerr << "error: unable to run model: " << e << std::endl;
    exit(1);
  }
  std::unique_ptr<tc::InferResult> r(result);
  FAIL_IF_ERR(result->RequestStatus(), "inference failed");
  if (verbose) std::cout << result->DebugString() << std::endl;
  example::ValidateSimple(result, d);
  tc::InferStat st;
  client->ClientInferStat(&st);
  std::cout << "completed " << st.completed_request_count << " requests" << std::endl;
  std::cout << "PASS : Infer" << std::endl;
  return 0;
}

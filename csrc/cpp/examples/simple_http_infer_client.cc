// Sync HTTP inference on `simple` (reference src/c++/examples/simple_http_infer_client.cc).
#include <getopt.h>

#include "example_util.h"
#include "http_client.h"

namespace tc = triton::client;

int main(int argc, char** argv)
{
  bool verbose = false;
  std::string url("localhost:8000");
  tc::Headers headers;
  tc::InferenceServerHttpClient::CompressionType req_comp = tc::InferenceServerHttpClient::CompressionType::NONE;
  tc::InferenceServerHttpClient::CompressionType resp_comp = tc::InferenceServerHttpClient::CompressionType::NONE;
  tc::HttpSslOptions ssl_options;
  // TLS flags of the reference example (an https:// URL turns TLS on)
  static const struct option longopts[] = {{"verify-peer", required_argument, nullptr, 1000},
                                           {"verify-host", required_argument, nullptr, 1001},
                                           {"ca-certs", required_argument, nullptr, 1002},
                                           {"cert-file", required_argument, nullptr, 1003},
                                           {"key-file", required_argument, nullptr, 1004},
                                           {nullptr, 0, nullptr, 0}};
  int opt;
  while ((opt = getopt_long(argc, argv, "vu:H:i:o:", longopts, nullptr)) != -1) {
    switch (opt) {
      case 1000: ssl_options.verify_peer = std::stol(optarg); break;
      case 1001: ssl_options.verify_host = std::stol(optarg); break;
      case 1002: ssl_options.ca_info = optarg; break;
      case 1003: ssl_options.cert = optarg; break;
      case 1004: ssl_options.key = optarg; break;
      case 'v': verbose = true; break;
      case 'u': url = optarg; break;
      case 'H': example::AddHeader(&headers, optarg); break;
      case 'i':
      case 'o': {
        std::string a = optarg;
        auto c = a == "gzip" ? tc::InferenceServerHttpClient::CompressionType::GZIP
                 : a == "deflate" ? tc::InferenceServerHttpClient::CompressionType::DEFLATE
                                  : tc::InferenceServerHttpClient::CompressionType::NONE;
        (opt == 'i' ? req_comp : resp_comp) = c;
        break;
      }
      default:
        example::Usage(argv, "\t-i <request compression: gzip|deflate>\n\t-o <response compression>\n"
                             "\t--verify-peer <0|1> --verify-host <0|2> --ca-certs <pem> --cert-file <pem> "
                             "--key-file <pem>");
    }
  }
  std::unique_ptr<tc::InferenceServerHttpClient> client;
  FAIL_IF_ERR(tc::InferenceServerHttpClient::Create(&client, url, verbose, ssl_options),
              "unable to create http client");
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
  options.request_id_ = "my_request";
  tc::InferResult* result;
  FAIL_IF_ERR(client->Infer(&result, options, {in0, in1}, {o0, o1}, headers, tc::Parameters(), req_comp, resp_comp),
              "unable to run model");
  std::unique_ptr<tc::InferResult> r(result);
  FAIL_IF_ERR(result->RequestStatus(), "inference failed");
  std::string id;
  result->Id(&id);
  if (id != "my_request") {
    std::cerr << "error: unexpected request id '" << id << "'" << std::endl;
    exit(1);
  }
  example::ValidateSimple(result, d);
  // JSON (non-binary) output for OUTPUT1
  o1->SetBinaryData(false);
  FAIL_IF_ERR(client->Infer(&result, options, {in0, in1}, {o0, o1}, headers), "unable to run model (json output)");
  r.reset(result);
  example::ValidateSimple(result, d, false);
  tc::InferStat st;
  client->ClientInferStat(&st);
  std::cout << "completed " << st.completed_request_count << " requests" << std::endl;
  std::cout << "PASS : Infer" << std::endl;
  return 0;
}

// Two sequences over one gRPC bidirectional stream, int and string
// correlation ids (reference src/c++/examples/simple_grpc_sequence_stream_infer_client.cc).
#include <getopt.h>

#include <condition_variable>
#include <map>
#include <mutex>

#include "example_util.h"
#include "grpc_client.h"

namespace tc = triton::client;

int main(int argc, char** argv)
{
  bool verbose = false, dyna = false;
  std::string url("localhost:8001");
  uint32_t stream_timeout = 0;
  int opt;
  while ((opt = getopt(argc, argv, "vdu:t:")) != -1) {
    switch (opt) {
      case 'v': verbose = true; break;
      case 'd': dyna = true; break;
      case 'u': url = optarg; break;
      case 't': stream_timeout = std::stoul(optarg); break;
      default: example::Usage(argv, "\t-d use simple_dyna_sequence\n\t-t <stream timeout us>");
    }
  }
  const std::string model = dyna ? "simple_dyna_sequence" : "simple_sequence";
  std::unique_ptr<tc::InferenceServerGrpcClient> client;
  FAIL_IF_ERR(tc::InferenceServerGrpcClient::Create(&client, url, verbose), "unable to create grpc client");
  std::mutex mu;
  std::condition_variable cv;
  std::map<std::string, int32_t> got;
  FAIL_IF_ERR(client->StartStream(
                  [&](tc::InferResult* r) {
                    std::unique_ptr<tc::InferResult> rr(r);
                    std::string id;
                    r->Id(&id);
                    int32_t v = -999999;
                    const uint8_t* buf;
                    size_t n;
                    if (r->RequestStatus().IsOk() && r->RawData("OUTPUT", &buf, &n).IsOk())
                      v = *reinterpret_cast<const int32_t*>(buf);
                    std::lock_guard<std::mutex> lk(mu);
                    got[id] = v;
                    cv.notify_all();
                  },
                  true, stream_timeout),
              "unable to start stream");
  const std::vector<int32_t> values = {11, 7, 5, 3, 2, 0, 1};
  std::vector<std::unique_ptr<tc::InferInput>> keep;
  std::vector<std::unique_ptr<int32_t>> data;  // input buffers must outlive the requests
  int sent = 0;
  for (int pass = 0; pass < 2; ++pass) {  // pass 0: int ids, pass 1: string ids
    for (int s = 0; s < 2; ++s) {
      for (size_t i = 0; i < values.size(); ++i) {
        tc::InferInput* in;
        FAIL_IF_ERR(tc::InferInput::Create(&in, "INPUT", {1, 1}, "INT32"), "unable to create INPUT");
        keep.emplace_back(in);
        data.emplace_back(new int32_t((s ? -1 : 1) * values[i]));
        int32_t* v = data.back().get();
        FAIL_IF_ERR(in->AppendRaw(reinterpret_cast<uint8_t*>(v), 4), "unable to set INPUT");
        tc::InferOptions options(model);
        if (pass == 0) options.sequence_id_ = 1000 + s;
        else options.sequence_id_str_ = "seq_" + std::to_string(s);
        options.sequence_start_ = i == 0;
        options.sequence_end_ = i + 1 == values.size();
        options.request_id_ = std::to_string(pass) + "_" + std::to_string(s) + "_" + std::to_string(i);
        FAIL_IF_ERR(client->AsyncStreamInfer(options, {in}), "unable to send stream request");
        ++sent;
      }
    }
  }
  {
    std::unique_lock<std::mutex> lk(mu);
    if (!cv.wait_for(lk, std::chrono::seconds(60), [&] { return (int)got.size() == sent; })) {
      std::cerr << "error: timed out, got " << got.size() << " of " << sent << " responses" << std::endl;
      exit(1);
    }
  }
  client->StopStream();
  for (auto& kv : got) {
    if (kv.second == -999999) {
      std::cerr << "error: request " << kv.first << " failed" << std::endl;
      exit(1);
    }
  }
  std::cout << "received " << got.size() << " responses" << std::endl;
  std::cout << "PASS : Sequence Stream" << std::endl;
  return 0;
}

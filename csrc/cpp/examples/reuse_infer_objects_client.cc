// Reuse InferInput / InferRequestedOutput across requests, switching between
// in-band tensors and system shared memory (Reset / UnsetSharedMemory), for
// HTTP and gRPC (reference src/c++/examples/reuse_infer_objects_client.cc).
#include <getopt.h>

#include "example_util.h"
#include "grpc_client.h"
#include "http_client.h"
#include "shm_utils.h"

namespace tc = triton::client;

template <typename Client>
static void Run(Client* client, const std::string& tag)
{
  example::SimpleData d;
  const size_t nbytes = 64;
  tc::InferInput *in0, *in1;
  FAIL_IF_ERR(tc::InferInput::Create(&in0, "INPUT0", {1, 16}, "INT32"), "INPUT0");
  FAIL_IF_ERR(tc::InferInput::Create(&in1, "INPUT1", {1, 16}, "INT32"), "INPUT1");
  std::unique_ptr<tc::InferInput> p0(in0), p1(in1);
  tc::InferRequestedOutput *o0, *o1;
  FAIL_IF_ERR(tc::InferRequestedOutput::Create(&o0, "OUTPUT0"), "OUTPUT0");
  FAIL_IF_ERR(tc::InferRequestedOutput::Create(&o1, "OUTPUT1"), "OUTPUT1");
  std::unique_ptr<tc::InferRequestedOutput> q0(o0), q1(o1);
  tc::InferOptions options("simple");
  // shared memory regions
  const std::string ik = "/reuse_in_" + tag + std::to_string(getpid()), ok = "/reuse_out_" + tag + std::to_string(getpid());
  int ifd, ofd;
  void *ia, *oa;
  FAIL_IF_ERR(tc::CreateSharedMemoryRegion(ik, nbytes * 2, &ifd), "create in");
  FAIL_IF_ERR(tc::MapSharedMemory(ifd, 0, nbytes * 2, &ia), "map in");
  FAIL_IF_ERR(tc::CreateSharedMemoryRegion(ok, nbytes * 2, &ofd), "create out");
  FAIL_IF_ERR(tc::MapSharedMemory(ofd, 0, nbytes * 2, &oa), "map out");
  memcpy(ia, d.in0.data(), nbytes);
  memcpy(static_cast<uint8_t*>(ia) + nbytes, d.in1.data(), nbytes);
  FAIL_IF_ERR(client->RegisterSystemSharedMemory("input_data", ik, nbytes * 2), "register in");
  FAIL_IF_ERR(client->RegisterSystemSharedMemory("output_data", ok, nbytes * 2), "register out");
  for (int round = 0; round < 3; ++round) {
    // round 0 / 2: in-band; round 1: shared memory (same objects)
    in0->Reset();
    in1->Reset();
    if (round == 1) {
      in0->SetSharedMemory("input_data", nbytes, 0);
      in1->SetSharedMemory("input_data", nbytes, nbytes);
      o0->SetSharedMemory("output_data", nbytes, 0);
      o1->SetSharedMemory("output_data", nbytes, nbytes);
    } else {
      in0->AppendRaw(reinterpret_cast<uint8_t*>(d.in0.data()), nbytes);
      in1->AppendRaw(reinterpret_cast<uint8_t*>(d.in1.data()), nbytes);
      o0->UnsetSharedMemory();
      o1->UnsetSharedMemory();
    }
    tc::InferResult* result;
    FAIL_IF_ERR(client->Infer(&result, options, {in0, in1}, {o0, o1}), "unable to run model");
    std::unique_ptr<tc::InferResult> r(result);
    FAIL_IF_ERR(result->RequestStatus(), "inference failed");
    if (round == 1) {
      const int32_t* s = static_cast<const int32_t*>(oa);
      for (int i = 0; i < 16; ++i)
        if (s[i] != d.in0[i] + d.in1[i] || s[16 + i] != d.in0[i] - d.in1[i]) {
          std::cerr << "error: incorrect shared memory result" << std::endl;
          exit(1);
        }
    } else {
      example::ValidateSimple(result, d, false);
    }
  }
  FAIL_IF_ERR(client->UnregisterSystemSharedMemory(), "unregister");
  tc::UnmapSharedMemory(ia, nbytes * 2);
  tc::UnmapSharedMemory(oa, nbytes * 2);
  tc::CloseSharedMemory(ifd);
  tc::CloseSharedMemory(ofd);
  tc::UnlinkSharedMemoryRegion(ik);
  tc::UnlinkSharedMemoryRegion(ok);
}

int main(int argc, char** argv)
{
  bool verbose = false;
  std::string url;
  std::string protocol = "http";
  int opt;
  while ((opt = getopt(argc, argv, "vu:i:")) != -1) {
    switch (opt) {
      case 'v': verbose = true; break;
      case 'u': url = optarg; break;
      case 'i': protocol = optarg; break;
      default: example::Usage(argv, "\t-i <http|grpc>");
    }
  }
  for (auto& ch : protocol) ch = static_cast<char>(tolower(ch));
  if (protocol == "grpc") {
    std::unique_ptr<tc::InferenceServerGrpcClient> client;
    FAIL_IF_ERR(tc::InferenceServerGrpcClient::Create(&client, url.empty() ? "localhost:8001" : url, verbose),
                "unable to create grpc client");
    Run(client.get(), "grpc");
  } else {
    std::unique_ptr<tc::InferenceServerHttpClient> client;
    FAIL_IF_ERR(tc::InferenceServerHttpClient::Create(&client, url.empty() ? "localhost:8000" : url, verbose),
                "unable to create http client");
    Run(client.get(), "http");
  }
  std::cout << "PASS : Reuse Infer Objects" << std::endl;
  return 0;
}

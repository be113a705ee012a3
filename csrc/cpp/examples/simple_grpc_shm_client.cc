// System shared memory for inputs and outputs over gRPC (reference
// src/c++/examples/simple_grpc_shm_client.cc).
#include <getopt.h>
#include <sys/mman.h>

#include "example_util.h"
#include "grpc_client.h"
#include "shm_utils.h"

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
  FAIL_IF_ERR(tc::InferenceServerGrpcClient::Create(&client, url, verbose), "unable to create grpc client");
  FAIL_IF_ERR(client->UnregisterSystemSharedMemory(), "unable to unregister all system shared memory regions");
  const size_t nbytes = 64;
  int in_fd, out_fd;
  void *in_addr, *out_addr;
  const std::string in_key = "/input_simple_" + std::to_string(getpid()), out_key = "/output_simple_" + std::to_string(getpid());
  FAIL_IF_ERR(tc::CreateSharedMemoryRegion(in_key, nbytes * 2, &in_fd), "unable to create input region");
  FAIL_IF_ERR(tc::MapSharedMemory(in_fd, 0, nbytes * 2, &in_addr), "unable to map input region");
  FAIL_IF_ERR(tc::CreateSharedMemoryRegion(out_key, nbytes * 2, &out_fd), "unable to create output region");
  FAIL_IF_ERR(tc::MapSharedMemory(out_fd, 0, nbytes * 2, &out_addr), "unable to map output region");
  example::SimpleData d;
  memcpy(in_addr, d.in0.data(), nbytes);
  memcpy(static_cast<uint8_t*>(in_addr) + nbytes, d.in1.data(), nbytes);
  FAIL_IF_ERR(client->RegisterSystemSharedMemory("input_data", in_key, nbytes * 2), "unable to register input");
  FAIL_IF_ERR(client->RegisterSystemSharedMemory("output_data", out_key, nbytes * 2), "unable to register output");
  tc::InferInput *in0, *in1;
  FAIL_IF_ERR(tc::InferInput::Create(&in0, "INPUT0", {1, 16}, "INT32"), "unable to get INPUT0");
  FAIL_IF_ERR(tc::InferInput::Create(&in1, "INPUT1", {1, 16}, "INT32"), "unable to get INPUT1");
  std::unique_ptr<tc::InferInput> p0(in0), p1(in1);
  FAIL_IF_ERR(in0->SetSharedMemory("input_data", nbytes, 0), "unable to set shm for INPUT0");
  FAIL_IF_ERR(in1->SetSharedMemory("input_data", nbytes, nbytes), "unable to set shm for INPUT1");
  tc::InferRequestedOutput *o0, *o1;
  FAIL_IF_ERR(tc::InferRequestedOutput::Create(&o0, "OUTPUT0"), "unable to get OUTPUT0");
  FAIL_IF_ERR(tc::InferRequestedOutput::Create(&o1, "OUTPUT1"), "unable to get OUTPUT1");
  std::unique_ptr<tc::InferRequestedOutput> q0(o0), q1(o1);
  FAIL_IF_ERR(o0->SetSharedMemory("output_data", nbytes, 0), "unable to set shm for OUTPUT0");
  FAIL_IF_ERR(o1->SetSharedMemory("output_data", nbytes, nbytes), "unable to set shm for OUTPUT1");
  tc::InferOptions options("simple");
  tc::InferResult* result;
  FAIL_IF_ERR(client->Infer(&result, options, {in0, in1}, {o0, o1}), "unable to run model");
  std::unique_ptr<tc::InferResult> r(result);
  FAIL_IF_ERR(result->RequestStatus(), "inference failed");
  const int32_t* s = static_cast<const int32_t*>(out_addr);
  const int32_t* df = s + 16;
  for (int i = 0; i < 16; ++i) {
    std::cout << d.in0[i] << " + " << d.in1[i] << " = " << s[i] << std::endl;
    std::cout << d.in0[i] << " - " << d.in1[i] << " = " << df[i] << std::endl;
    if (d.in0[i] + d.in1[i] != s[i] || d.in0[i] - d.in1[i] != df[i]) {
      std::cerr << "error: incorrect result" << std::endl;
      exit(1);
    }
  }
  inference::SystemSharedMemoryStatusResponse status;
  FAIL_IF_ERR(client->SystemSharedMemoryStatus(&status), "unable to get shared memory status");
  std::cout << "Shared Memory Status:\n" << status.DebugString() << std::endl;
  FAIL_IF_ERR(client->UnregisterSystemSharedMemory(), "unable to unregister shared memory");
  tc::UnmapSharedMemory(in_addr, nbytes * 2);
  tc::UnmapSharedMemory(out_addr, nbytes * 2);
  tc::CloseSharedMemory(in_fd);
  tc::CloseSharedMemory(out_fd);
  tc::UnlinkSharedMemoryRegion(in_key);
  tc::UnlinkSharedMemoryRegion(out_key);
  std::cout << "PASS : System Shared Memory " << std::endl;
  return 0;
}

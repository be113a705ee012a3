// Device (HIP) shared memory over HTTP: inputs and outputs in GPU memory
// registered by IPC handle (reference src/c++/examples/simple_http_cudashm_client.cc;
// cudaIpcMemHandle_t is hipIpcMemHandle_t on MI355X, see include/ipc.h).
#include <getopt.h>
#include <hip/hip_runtime_api.h>

#include "example_util.h"
#include "http_client.h"

namespace tc = triton::client;

#define FAIL_IF_HIP_ERR(X, MSG)                                                  \
  do {                                                                           \
    hipError_t e__ = (X);                                                        \
    if (e__ != hipSuccess) {                                                     \
      std::cerr << "error: " << (MSG) << ": " << hipGetErrorString(e__) << std::endl; \
      exit(1);                                                                   \
    }                                                                            \
  } while (false)

int main(int argc, char** argv)
{
  bool verbose = false;
  std::string url("localhost:8000");
  int device = 0;
  int opt;
  while ((opt = getopt(argc, argv, "vu:d:")) != -1) {
    switch (opt) {
      case 'v': verbose = true; break;
      case 'u': url = optarg; break;
      case 'd': device = std::stoi(optarg); break;
      default: example::Usage(argv, "\t-d <device id>");
    }
  }
  std::unique_ptr<tc::InferenceServerHttpClient> client;
  FAIL_IF_ERR(tc::InferenceServerHttpClient::Create(&client, url, verbose), "unable to create client");
  FAIL_IF_ERR(client->UnregisterCudaSharedMemory(), "unable to unregister device regions");
  const size_t nbytes = 64;
  example::SimpleData d;
  FAIL_IF_HIP_ERR(hipSetDevice(device), "hipSetDevice");
  void *in_d, *out_d;
  FAIL_IF_HIP_ERR(hipMalloc(&in_d, nbytes * 2), "hipMalloc input");
  FAIL_IF_HIP_ERR(hipMalloc(&out_d, nbytes * 2), "hipMalloc output");
  FAIL_IF_HIP_ERR(hipMemcpy(in_d, d.in0.data(), nbytes, hipMemcpyHostToDevice), "copy INPUT0");
  FAIL_IF_HIP_ERR(hipMemcpy(static_cast<uint8_t*>(in_d) + nbytes, d.in1.data(), nbytes, hipMemcpyHostToDevice),
                  "copy INPUT1");
  cudaIpcMemHandle_t in_h, out_h;
  FAIL_IF_HIP_ERR(hipIpcGetMemHandle(&in_h, in_d), "ipc handle input");
  FAIL_IF_HIP_ERR(hipIpcGetMemHandle(&out_h, out_d), "ipc handle output");
  FAIL_IF_ERR(client->RegisterCudaSharedMemory("input_data", in_h, device, nbytes * 2), "register input");
  FAIL_IF_ERR(client->RegisterCudaSharedMemory("output_data", out_h, device, nbytes * 2), "register output");
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
  int32_t out[32];
  FAIL_IF_HIP_ERR(hipMemcpy(out, out_d, nbytes * 2, hipMemcpyDeviceToHost), "copy outputs");
  for (int i = 0; i < 16; ++i) {
    std::cout << d.in0[i] << " + " << d.in1[i] << " = " << out[i] << std::endl;
    std::cout << d.in0[i] << " - " << d.in1[i] << " = " << out[16 + i] << std::endl;
    if (d.in0[i] + d.in1[i] != out[i] || d.in0[i] - d.in1[i] != out[16 + i]) {
      std::cerr << "error: incorrect result" << std::endl;
      exit(1);
    }
  }
  FAIL_IF_ERR(client->UnregisterCudaSharedMemory(), "unable to unregister device regions");
  FAIL_IF_HIP_ERR(hipFree(in_d), "hipFree");
  FAIL_IF_HIP_ERR(hipFree(out_d), "hipFree");
  std::cout << "PASS : Cuda Shared Memory " << std::endl;
  return 0;
}

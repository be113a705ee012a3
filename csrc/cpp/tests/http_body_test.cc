// http_body_test: sends the two request bodies whose base64 framing is a
// reference wire quirk (libb64, src/c++/library/cencode.c:78-81,106) to a URL
// given on the command line, for tests/test_cpp_examples.py to capture and
// compare byte for byte:
//   1. LoadModel("b64_model", config "{}", files {"file:1/model.onnx": bytes
//      0..N-1 mod 251}) for N = argv[2] (default 200)
//   2. RegisterCudaSharedMemory("b64_region", handle bytes 0..63, device 0,
//      byte size 4096)
// Exit status 0 when both calls returned (any HTTP status is fine: the
// capture side answers 200 "{}").
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <map>
#include <string>
#include <vector>

#include "http_client.h"

namespace tc = triton::client;

int
main(int argc, char** argv)
{
  if (argc < 2) {
    std::cerr << "usage: http_body_test host:port [file_bytes]" << std::endl;
    return 2;
  }
  const size_t n = argc > 2 ? static_cast<size_t>(std::atol(argv[2])) : 200;
  std::unique_ptr<tc::InferenceServerHttpClient> c;
  tc::Error e = tc::InferenceServerHttpClient::Create(&c, argv[1]);
  if (!e.IsOk()) {
    std::cerr << "create: " << e << std::endl;
    return 1;
  }
  std::vector<char> content(n);
  for (size_t i = 0; i < n; ++i) content[i] = static_cast<char>(i % 251);
  std::map<std::string, std::vector<char>> files{{"file:1/model.onnx", content}};
  e = c->LoadModel("b64_model", tc::Headers(), tc::Parameters(), "{}", files);
  if (!e.IsOk()) {
    std::cerr << "load: " << e << std::endl;
    return 1;
  }
  cudaIpcMemHandle_t h;
  unsigned char raw[sizeof(h)];
  for (size_t i = 0; i < sizeof(h); ++i) raw[i] = static_cast<unsigned char>(i);
  std::memcpy(&h, raw, sizeof(h));
  e = c->RegisterCudaSharedMemory("b64_region", h, 0, 4096);
  if (!e.IsOk()) {
    std::cerr << "register: " << e << std::endl;
    return 1;
  }
  return 0;
}

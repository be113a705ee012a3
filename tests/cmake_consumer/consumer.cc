// add/sub through both protocols, linked from an installed TritonClient package.
#include <iostream>
#include <memory>
#include <vector>

#include "grpc_client.h"
#include "http_client.h"

namespace tc = triton::client;

template <typename Client>
static int
Run(Client* c, const char* kind)
{
  std::vector<int32_t> a(16), b(16, 1);
  for (int i = 0; i < 16; ++i) a[i] = i;
  tc::InferInput *i0, *i1;
  tc::InferInput::Create(&i0, "INPUT0", {1, 16}, "INT32");
  tc::InferInput::Create(&i1, "INPUT1", {1, 16}, "INT32");
  std::unique_ptr<tc::InferInput> o0(i0), o1(i1);
  i0->AppendRaw(reinterpret_cast<uint8_t*>(a.data()), 64);
  i1->AppendRaw(reinterpret_cast<uint8_t*>(b.data()), 64);
  tc::InferResult* r = nullptr;
  tc::Error err = c->Infer(&r, tc::InferOptions("simple"), {i0, i1});
  if (!err.IsOk()) {
    std::cerr << kind << ": " << err.Message() << std::endl;
    return 1;
  }
  std::unique_ptr<tc::InferResult> own(r);
  const uint8_t* buf;
  size_t n;
  r->RawData("OUTPUT0", &buf, &n);
  const int32_t* s = reinterpret_cast<const int32_t*>(buf);
  for (int i = 0; i < 16; ++i)
    if (s[i] != i + 1) return 1;
  std::cout << kind << " ok" << std::endl;
  return 0;
}

int
main(int argc, char** argv)
{
  if (argc < 3) return 2;
  std::unique_ptr<tc::InferenceServerHttpClient> http;
  std::unique_ptr<tc::InferenceServerGrpcClient> grpc;
  if (!tc::InferenceServerHttpClient::Create(&http, argv[1]).IsOk()) return 1;
  if (!tc::InferenceServerGrpcClient::Create(&grpc, argv[2]).IsOk()) return 1;
  return Run(http.get(), "http") | Run(grpc.get(), "grpc");
}

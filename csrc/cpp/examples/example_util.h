// Shared helpers of the C++ examples (ports of reference src/c++/examples/*).
#pragma once

#include <unistd.h>

#include <cstdint>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "common.h"

#define FAIL_IF_ERR(X, MSG)                                          \
  do {                                                               \
    triton::client::Error err__ = (X);                               \
    if (!err__.IsOk()) {                                             \
      std::cerr << "error: " << (MSG) << ": " << err__ << std::endl; \
      exit(1);                                                       \
    }                                                                \
  } while (false)

namespace example {

inline void Usage(char** argv, const std::string& extra = "")
{
  std::cerr << "Usage: " << argv[0] << " [options]" << std::endl
            << "\t-v verbose" << std::endl
            << "\t-u <URL for inference service>" << std::endl
            << "\t-H <HTTP header / gRPC metadata 'Name:Value'>" << std::endl
            << extra << std::endl;
  exit(1);
}

/// INPUT0 = 0..15, INPUT1 = 1 (the `simple` model's standard request).
struct SimpleData {
  std::vector<int32_t> in0, in1;
  SimpleData()
  {
    for (int i = 0; i < 16; ++i) {
      in0.push_back(i);
      in1.push_back(1);
    }
  }
};

/// Check OUTPUT0 = INPUT0 + INPUT1 and OUTPUT1 = INPUT0 - INPUT1 of a result.
inline void ValidateSimple(triton::client::InferResult* result, const SimpleData& d, bool print = true)
{
  std::vector<int64_t> shape;
  std::string dt;
  FAIL_IF_ERR(result->Shape("OUTPUT0", &shape), "unable to get shape for 'OUTPUT0'");
  if (shape.size() != 2 || shape[0] != 1 || shape[1] != 16) {
    std::cerr << "error: received incorrect shapes for 'OUTPUT0'" << std::endl;
    exit(1);
  }
  FAIL_IF_ERR(result->Datatype("OUTPUT0", &dt), "unable to get datatype for 'OUTPUT0'");
  if (dt != "INT32") {
    std::cerr << "error: received incorrect datatype for 'OUTPUT0': " << dt << std::endl;
    exit(1);
  }
  const uint8_t *b0, *b1;
  size_t n0, n1;
  FAIL_IF_ERR(result->RawData("OUTPUT0", &b0, &n0), "unable to get result data for 'OUTPUT0'");
  FAIL_IF_ERR(result->RawData("OUTPUT1", &b1, &n1), "unable to get result data for 'OUTPUT1'");
  if (n0 != 64 || n1 != 64) {
    std::cerr << "error: received incorrect byte size for outputs: " << n0 << ", " << n1 << std::endl;
    exit(1);
  }
  const int32_t* s = reinterpret_cast<const int32_t*>(b0);
  const int32_t* df = reinterpret_cast<const int32_t*>(b1);
  for (int i = 0; i < 16; ++i) {
    if (print) {
      std::cout << d.in0[i] << " + " << d.in1[i] << " = " << s[i] << std::endl;
      std::cout << d.in0[i] << " - " << d.in1[i] << " = " << df[i] << std::endl;
    }
    if (d.in0[i] + d.in1[i] != s[i] || d.in0[i] - d.in1[i] != df[i]) {
      std::cerr << "error: incorrect result" << std::endl;
      exit(1);
    }
  }
}

/// Parse one -H 'Name:Value' argument into the header map.
template <typename Map>
inline void AddHeader(Map* headers, const std::string& arg)
{
  auto p = arg.find(':');
  if (p == std::string::npos) {
    std::cerr << "error: -H expects Name:Value" << std::endl;
    exit(1);
  }
  (*headers)[arg.substr(0, p)] = arg.substr(p + 1);
}

}  // namespace example

// InferenceServerHttpClient — KServe-v2 REST client for MI355X hosts.
//
// API parity with reference src/c++/library/http_client.h:38-649 (same class,
// method names, argument order and defaults).  Transport is new: no libcurl.
//  * sync calls use a blocking keep-alive HTTP/1.1 connection per client;
//  * AsyncInfer runs an epoll event loop on one worker thread that owns a pool
//    of non-blocking connections (one request in flight per connection), and
//    sends each request with writev() straight from the user's InferInput
//    buffers — the JSON header and tensors are never concatenated;
//  * gzip/deflate via zlib, TLS via OpenSSL.
#pragma once

#include <atomic>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "common.h"
#include "ipc.h"

namespace triton { namespace client {

using Headers = std::map<std::string, std::string>;
using Parameters = std::map<std::string, std::string>;

struct HttpSslOptions {
  enum CERTTYPE { CERT_PEM = 0, CERT_DER = 1 };
  enum KEYTYPE { KEY_PEM = 0, KEY_DER = 1 };
  explicit HttpSslOptions()
      : verify_peer(1), verify_host(2), cert_type(CERTTYPE::CERT_PEM), key_type(KEYTYPE::KEY_PEM)
  {
  }
  long verify_peer;
  long verify_host;
  std::string ca_info;
  CERTTYPE cert_type;
  std::string cert;
  KEYTYPE key_type;
  std::string key;
};

class HttpConnection;
class HttpAsyncEngine;
struct HttpPreparedRequest;

class InferenceServerHttpClient : public InferenceServerClient {
 public:
  enum class CompressionType { NONE, DEFLATE, GZIP };

  ~InferenceServerHttpClient();

  /// Build the request body: JSON header followed by binary inputs.
  static Error GenerateRequestBody(
      std::vector<char>* request_body, size_t* header_length, const InferOptions& options,
      const std::vector<InferInput*>& inputs,
      const std::vector<const InferRequestedOutput*>& outputs = std::vector<const InferRequestedOutput*>());

  /// Parse a response body (header_length 0 = whole body is JSON).
  static Error ParseResponseBody(
      InferResult** result, const std::vector<char>& response_body, const size_t header_length = 0);

  static Error Create(
      std::unique_ptr<InferenceServerHttpClient>* client, const std::string& server_url, bool verbose = false,
      const HttpSslOptions& ssl_options = HttpSslOptions());

  Error IsServerLive(bool* live, const Headers& headers = Headers(), const Parameters& query_params = Parameters());
  Error IsServerReady(bool* ready, const Headers& headers = Headers(), const Parameters& query_params = Parameters());
  Error IsModelReady(
      bool* ready, const std::string& model_name, const std::string& model_version = "",
      const Headers& headers = Headers(), const Parameters& query_params = Parameters());
  Error ServerMetadata(
      std::string* server_metadata, const Headers& headers = Headers(), const Parameters& query_params = Parameters());
  Error ModelMetadata(
      std::string* model_metadata, const std::string& model_name, const std::string& model_version = "",
      const Headers& headers = Headers(), const Parameters& query_params = Parameters());
  Error ModelConfig(
      std::string* model_config, const std::string& model_name, const std::string& model_version = "",
      const Headers& headers = Headers(), const Parameters& query_params = Parameters());
  Error ModelRepositoryIndex(
      std::string* repository_index, const Headers& headers = Headers(), const Parameters& query_params = Parameters());
  Error LoadModel(
      const std::string& model_name, const Headers& headers = Headers(), const Parameters& query_params = Parameters(),
      const std::string& config = std::string(), const std::map<std::string, std::vector<char>>& files = {});
  Error UnloadModel(
      const std::string& model_name, const Headers& headers = Headers(), const Parameters& query_params = Parameters());
  Error ModelInferenceStatistics(
      std::string* infer_stat, const std::string& model_name = "", const std::string& model_version = "",
      const Headers& headers = Headers(), const Parameters& query_params = Parameters());
  Error UpdateTraceSettings(
      std::string* response, const std::string& model_name = "",
      const std::map<std::string, std::vector<std::string>>& settings = std::map<std::string, std::vector<std::string>>(),
      const Headers& headers = Headers(), const Parameters& query_params = Parameters());
  Error GetTraceSettings(
      std::string* settings, const std::string& model_name = "", const Headers& headers = Headers(),
      const Parameters& query_params = Parameters());
  Error UpdateLogSettings(
      std::string* response, const std::map<std::string, std::string>& settings, const Headers& headers = Headers(),
      const Parameters& query_params = Parameters());
  Error GetLogSettings(
      std::string* settings, const Headers& headers = Headers(), const Parameters& query_params = Parameters());
  Error SystemSharedMemoryStatus(
      std::string* status, const std::string& region_name = "", const Headers& headers = Headers(),
      const Parameters& query_params = Parameters());
  Error RegisterSystemSharedMemory(
      const std::string& name, const std::string& key, const size_t byte_size, const size_t offset = 0,
      const Headers& headers = Headers(), const Parameters& query_params = Parameters());
  Error UnregisterSystemSharedMemory(
      const std::string& name = "", const Headers& headers = Headers(), const Parameters& query_params = Parameters());
  Error CudaSharedMemoryStatus(
      std::string* status, const std::string& region_name = "", const Headers& headers = Headers(),
      const Parameters& query_params = Parameters());
  /// Register a device region by its 64-byte IPC handle (hipIpcMemHandle_t).
  Error RegisterCudaSharedMemory(
      const std::string& name, const cudaIpcMemHandle_t& cuda_shm_handle, const size_t device_id,
      const size_t byte_size, const Headers& headers = Headers(), const Parameters& query_params = Parameters());
  Error UnregisterCudaSharedMemory(
      const std::string& name = "", const Headers& headers = Headers(), const Parameters& query_params = Parameters());

  Error Infer(
      InferResult** result, const InferOptions& options, const std::vector<InferInput*>& inputs,
      const std::vector<const InferRequestedOutput*>& outputs = std::vector<const InferRequestedOutput*>(),
      const Headers& headers = Headers(), const Parameters& query_params = Parameters(),
      const CompressionType request_compression_algorithm = CompressionType::NONE,
      const CompressionType response_compression_algorithm = CompressionType::NONE);

  Error AsyncInfer(
      OnCompleteFn callback, const InferOptions& options, const std::vector<InferInput*>& inputs,
      const std::vector<const InferRequestedOutput*>& outputs = std::vector<const InferRequestedOutput*>(),
      const Headers& headers = Headers(), const Parameters& query_params = Parameters(),
      const CompressionType request_compression_algorithm = CompressionType::NONE,
      const CompressionType response_compression_algorithm = CompressionType::NONE);

  Error InferMulti(
      std::vector<InferResult*>* results, const std::vector<InferOptions>& options,
      const std::vector<std::vector<InferInput*>>& inputs,
      const std::vector<std::vector<const InferRequestedOutput*>>& outputs =
          std::vector<std::vector<const InferRequestedOutput*>>(),
      const Headers& headers = Headers(), const Parameters& query_params = Parameters(),
      const CompressionType request_compression_algorithm = CompressionType::NONE,
      const CompressionType response_compression_algorithm = CompressionType::NONE);

  Error AsyncInferMulti(
      OnMultiCompleteFn callback, const std::vector<InferOptions>& options,
      const std::vector<std::vector<InferInput*>>& inputs,
      const std::vector<std::vector<const InferRequestedOutput*>>& outputs =
          std::vector<std::vector<const InferRequestedOutput*>>(),
      const Headers& headers = Headers(), const Parameters& query_params = Parameters(),
      const CompressionType request_compression_algorithm = CompressionType::NONE,
      const CompressionType response_compression_algorithm = CompressionType::NONE);

  /// Max concurrent async connections (default 256).
  void SetMaxAsyncConnections(size_t n) { max_async_conns_ = n; }

 private:
  InferenceServerHttpClient(const std::string& url, bool verbose, const HttpSslOptions& ssl_options);

  Error Get(std::string& request_uri, const Headers& headers, const Parameters& query_params, std::string* response,
            long* http_code = nullptr);
  Error Post(std::string& request_uri, const std::string& request, const Headers& headers,
             const Parameters& query_params, std::string* response, long* http_code = nullptr);
  Error Request(const std::string& method, std::string& uri, const std::vector<std::pair<const char*, size_t>>& body,
                const Headers& headers, const Parameters& query_params, long* http_code, std::string* response_body,
                std::map<std::string, std::string>* response_headers, uint64_t timeout_us,
                RequestTimers* timers = nullptr);
  Error PrepareInfer(
      const InferOptions& options, const std::vector<InferInput*>& inputs,
      const std::vector<const InferRequestedOutput*>& outputs, const Headers& headers, const Parameters& query_params,
      CompressionType request_compression, CompressionType response_compression, HttpPreparedRequest* req);

  friend class HttpAsyncEngine;
  std::string host_;
  int port_;
  std::string base_path_;
  bool use_ssl_;
  HttpSslOptions ssl_options_;
  std::unique_ptr<HttpConnection> sync_conn_;
  std::mutex sync_mu_;
  std::unique_ptr<HttpAsyncEngine> engine_;
  size_t max_async_conns_ = 256;
};

}}  // namespace triton::client

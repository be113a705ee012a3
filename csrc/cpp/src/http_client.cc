// InferenceServerHttpClient implementation (see include/http_client.h).
//
// Wire behaviour follows the reference client
// (src/c++/library/http_client.cc:411-578 request JSON, :1042-1281 response
// parsing, :1393-1764 control plane) with the documented bug fixes:
// IsServerReady hits /v2/health/ready (reference :1416 uses /live) and FP64
// JSON->binary conversion uses a double buffer (reference :1245 overflows).
#include "http_client.h"

#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <deque>
#include <iostream>
#include <unordered_map>

#include "json.h"
#include "net.h"
#include "trace.h"

namespace triton { namespace client {

using json::Value;
using K = RequestTimers::Kind;

//==============================================================================
// Result
//==============================================================================
namespace {

struct OutputEntry {
  std::string name, datatype;
  std::vector<int64_t> shape;
  const uint8_t* data = nullptr;
  size_t size = 0;
  bool has_data = false;
  std::string owned;  // converted JSON data
};

Error
JsonToBinary(const Value& data, const std::string& dt, std::string* out)
{
  out->clear();
  std::vector<const Value*> flat;
  std::function<void(const Value&)> walk = [&](const Value& v) {
    if (v.IsArray()) {
      for (const auto& e : v.Elements()) walk(e);
    } else {
      flat.push_back(&v);
    }
  };
  walk(data);
  auto put = [&](const void* p, size_t n) { out->append(static_cast<const char*>(p), n); };
  for (const Value* v : flat) {
    if (dt == "BOOL") { uint8_t x = v->AsBool(); put(&x, 1); }
    else if (dt == "INT8") { int8_t x = static_cast<int8_t>(v->AsInt()); put(&x, 1); }
    else if (dt == "INT16") { int16_t x = static_cast<int16_t>(v->AsInt()); put(&x, 2); }
    else if (dt == "INT32") { int32_t x = static_cast<int32_t>(v->AsInt()); put(&x, 4); }
    else if (dt == "INT64") { int64_t x = v->AsInt(); put(&x, 8); }
    else if (dt == "UINT8") { uint8_t x = static_cast<uint8_t>(v->AsUInt()); put(&x, 1); }
    else if (dt == "UINT16") { uint16_t x = static_cast<uint16_t>(v->AsUInt()); put(&x, 2); }
    else if (dt == "UINT32") { uint32_t x = static_cast<uint32_t>(v->AsUInt()); put(&x, 4); }
    else if (dt == "UINT64") { uint64_t x = v->AsUInt(); put(&x, 8); }
    else if (dt == "FP32") { float x = static_cast<float>(v->AsDouble()); put(&x, 4); }
    else if (dt == "FP64") { double x = v->AsDouble(); put(&x, 8); }
    else if (dt == "BYTES") {
      const std::string& s = v->AsString();
      uint32_t n = static_cast<uint32_t>(s.size());
      put(&n, 4);
      put(s.data(), s.size());
    } else {
      return Error("datatype '" + dt + "' is not supported in JSON output");
    }
  }
  return Error::Success;
}

class InferResultHttp : public InferResult {
 public:
  static Error Create(InferResult** result, std::string&& body, size_t header_length, long http_code,
                      const std::string& client_error)
  {
    auto* r = new InferResultHttp();
    r->body_ = std::move(body);
    r->Parse(header_length, http_code, client_error);
    *result = r;
    return Error::Success;
  }

  Error ModelName(std::string* name) const override { return Field("model_name", name); }
  Error ModelVersion(std::string* version) const override { return Field("model_version", version); }
  Error Id(std::string* id) const override { return Field("id", id); }
  Error Shape(const std::string& output_name, std::vector<int64_t>* shape) const override
  {
    const OutputEntry* o = Find(output_name);
    if (!o) return Error("The response does not contain results for output name '" + output_name + "'");
    *shape = o->shape;
    return Error::Success;
  }
  Error Datatype(const std::string& output_name, std::string* datatype) const override
  {
    const OutputEntry* o = Find(output_name);
    if (!o) return Error("The response does not contain results for output name '" + output_name + "'");
    *datatype = o->datatype;
    return Error::Success;
  }
  Error RawData(const std::string& output_name, const uint8_t** buf, size_t* byte_size) const override
  {
    const OutputEntry* o = Find(output_name);
    if (!o || !o->has_data) {
      return Error("The response does not contain results for output name '" + output_name + "'");
    }
    *buf = o->data;
    *byte_size = o->size;
    return Error::Success;
  }
  Error IsFinalResponse(bool* is_final_response) const override
  {
    *is_final_response = true;
    return Error::Success;
  }
  Error IsNullResponse(bool* is_null_response) const override
  {
    *is_null_response = false;
    return Error::Success;
  }
  Error StringData(const std::string& output_name, std::vector<std::string>* string_result) const override
  {
    std::string dt;
    Error e = Datatype(output_name, &dt);
    if (!e.IsOk()) return e;
    if (dt != "BYTES") {
      return Error("This function supports tensors with datatype 'BYTES', requested output tensor '" +
                   output_name + "' with datatype '" + dt + "'");
    }
    const uint8_t* buf = nullptr;
    size_t n = 0;
    e = RawData(output_name, &buf, &n);
    if (!e.IsOk()) return e;
    string_result->clear();
    size_t pos = 0;
    while (pos + 4 <= n) {
      uint32_t len;
      std::memcpy(&len, buf + pos, 4);
      pos += 4;
      if (pos + len > n) return Error("malformed BYTES output '" + output_name + "'");
      string_result->emplace_back(reinterpret_cast<const char*>(buf + pos), len);
      pos += len;
    }
    return Error::Success;
  }
  std::string DebugString() const override { return header_.Serialize(); }
  Error RequestStatus() const override { return status_; }

 private:
  Error Field(const char* key, std::string* out) const
  {
    const Value* v = header_.IsObject() ? header_.Find(key) : nullptr;
    if (!v) return Error(std::string(key) + " was not returned in the response");
    *out = v->AsString();
    return Error::Success;
  }
  const OutputEntry* Find(const std::string& name) const
  {
    for (const auto& o : outputs_)
      if (o.name == name) return &o;
    return nullptr;
  }
  void Parse(size_t header_length, long http_code, const std::string& client_error)
  {
    if (!client_error.empty()) {
      status_ = Error(client_error);
      return;
    }
    if (http_code == 499) {
      status_ = Error("Deadline Exceeded");
      return;
    }
    size_t hl = header_length ? header_length : body_.size();
    if (hl > body_.size()) {
      status_ = Error("inference header length exceeds the response body");
      return;
    }
    std::string err;
    if (!json::Parse(body_.data(), hl, &header_, &err)) {
      status_ = Error("failed to parse the request JSON buffer: " + err);
      return;
    }
    if (http_code != 200) {
      const Value* e = header_.IsObject() ? header_.Find("error") : nullptr;
      status_ = Error(e ? e->AsString() : ("HTTP " + std::to_string(http_code)));
      return;
    }
    const Value* outs = header_.Find("outputs");
    size_t pos = hl;
    if (outs && outs->IsArray()) {
      for (const auto& o : outs->Elements()) {
        OutputEntry e;
        if (const Value* v = o.Find("name")) e.name = v->AsString();
        if (const Value* v = o.Find("datatype")) e.datatype = v->AsString();
        if (const Value* v = o.Find("shape"))
          for (const auto& d : v->Elements()) e.shape.push_back(d.AsInt());
        const Value* params = o.Find("parameters");
        const Value* bsz = params ? params->Find("binary_data_size") : nullptr;
        if (bsz) {
          e.size = bsz->AsUInt();
          if (pos + e.size > body_.size()) {
            status_ = Error("binary output '" + e.name + "' overruns the response body");
            return;
          }
          e.data = reinterpret_cast<const uint8_t*>(body_.data() + pos);
          e.has_data = true;
          pos += e.size;
        } else if (const Value* d = o.Find("data")) {
          Error ce = JsonToBinary(*d, e.datatype, &e.owned);
          if (!ce.IsOk()) {
            status_ = ce;
            return;
          }
          e.has_data = true;
        }
        outputs_.push_back(std::move(e));
      }
      // owned buffers are final now: take stable pointers
      for (auto& e : outputs_) {
        if (e.has_data && e.data == nullptr) {
          e.data = reinterpret_cast<const uint8_t*>(e.owned.data());
          e.size = e.owned.size();
        }
      }
    }
  }

  std::string body_;
  Value header_;
  std::vector<OutputEntry> outputs_;
  Error status_;
};

void
AppendHeaderLine(std::string* s, const std::string& k, const std::string& v)
{
  s->append(k);
  s->append(": ");
  s->append(v);
  s->append("\r\n");
}

std::string
QueryString(const Parameters& q)
{
  std::string s;
  for (const auto& kv : q) {
    s.append(s.empty() ? "?" : "&");
    s.append(UrlEncode(kv.first));
    s.push_back('=');
    s.append(UrlEncode(kv.second));
  }
  return s;
}

Error
InputToJson(InferInput* in, Value* data)
{
  const std::string& dt = in->Datatype();
  if (dt == "FP16" || dt == "BF16" || dt == "FP8_E4M3" || dt == "FP8_E5M2") {
    return Error("datatype '" + dt + "' of input '" + in->Name() + "' cannot be sent as JSON; use binary data");
  }
  std::string raw;
  for (size_t i = 0; i < in->Buffers().size(); ++i)
    raw.append(reinterpret_cast<const char*>(in->Buffers()[i]), in->BufferSizes()[i]);
  *data = Value::Array();
  const char* p = raw.data();
  size_t n = raw.size();
  auto each = [&](size_t es, auto fn) {
    if (n % es) return Error("input '" + in->Name() + "' byte size is not a multiple of the element size");
    for (size_t i = 0; i < n; i += es) fn(p + i);
    return Error::Success;
  };
  if (dt == "BOOL") return each(1, [&](const char* q) { data->Append(Value(*q != 0)); });
  if (dt == "INT8") return each(1, [&](const char* q) { data->Append(Value(static_cast<int64_t>(*reinterpret_cast<const int8_t*>(q)))); });
  if (dt == "UINT8") return each(1, [&](const char* q) { data->Append(Value(static_cast<uint64_t>(*reinterpret_cast<const uint8_t*>(q)))); });
  if (dt == "INT16") return each(2, [&](const char* q) { int16_t v; std::memcpy(&v, q, 2); data->Append(Value(static_cast<int64_t>(v))); });
  if (dt == "UINT16") return each(2, [&](const char* q) { uint16_t v; std::memcpy(&v, q, 2); data->Append(Value(static_cast<uint64_t>(v))); });
  if (dt == "INT32") return each(4, [&](const char* q) { int32_t v; std::memcpy(&v, q, 4); data->Append(Value(static_cast<int64_t>(v))); });
  if (dt == "UINT32") return each(4, [&](const char* q) { uint32_t v; std::memcpy(&v, q, 4); data->Append(Value(static_cast<uint64_t>(v))); });
  if (dt == "INT64") return each(8, [&](const char* q) { int64_t v; std::memcpy(&v, q, 8); data->Append(Value(v)); });
  if (dt == "UINT64") return each(8, [&](const char* q) { uint64_t v; std::memcpy(&v, q, 8); data->Append(Value(v)); });
  if (dt == "FP32") return each(4, [&](const char* q) { float v; std::memcpy(&v, q, 4); data->Append(Value(static_cast<double>(v))); });
  if (dt == "FP64") return each(8, [&](const char* q) { double v; std::memcpy(&v, q, 8); data->Append(Value(v)); });
  if (dt == "BYTES") {
    size_t pos = 0;
    while (pos + 4 <= n) {
      uint32_t len;
      std::memcpy(&len, p + pos, 4);
      pos += 4;
      if (pos + len > n) return Error("malformed BYTES input '" + in->Name() + "'");
      data->Append(Value(std::string(p + pos, len)));
      pos += len;
    }
    return Error::Success;
  }
  return Error("unknown datatype '" + dt + "'");
}

Error
BuildRequestJson(
    const InferOptions& options, const std::vector<InferInput*>& inputs,
    const std::vector<const InferRequestedOutput*>& outputs, std::string* out)
{
  Value req = Value::Object();
  req.Set("id", Value(options.request_id_));  // always present, like the reference C++ client
  Value params = Value::Object();
  if (options.sequence_id_ != 0 || !options.sequence_id_str_.empty()) {
    if (!options.sequence_id_str_.empty()) params.Set("sequence_id", Value(options.sequence_id_str_));
    else params.Set("sequence_id", Value(options.sequence_id_));
    params.Set("sequence_start", Value(options.sequence_start_));
    params.Set("sequence_end", Value(options.sequence_end_));
  }
  if (options.priority_ != 0) params.Set("priority", Value(options.priority_));
  if (options.server_timeout_ != 0) params.Set("timeout", Value(options.server_timeout_));
  if (outputs.empty()) params.Set("binary_data_output", Value(true));
  for (const auto& kv : options.request_parameters) {
    const RequestParameter& p = kv.second;
    if (p.name == "sequence_id" || p.name == "sequence_start" || p.name == "sequence_end" ||
        p.name == "priority" || p.name == "binary_data_output") {
      return Error("Parameter \"" + p.name + "\" is a reserved parameter and cannot be specified.");
    }
    if (p.type == "bool") params.Set(p.name, Value(p.value == "true" || p.value == "1"));
    else if (p.type == "int") params.Set(p.name, Value(static_cast<int64_t>(std::stoll(p.value))));
    else if (p.type == "double") params.Set(p.name, Value(std::stod(p.value)));
    else params.Set(p.name, Value(p.value));
  }
  if (params.Size()) req.Set("parameters", std::move(params));
  Value ins = Value::Array();
  for (InferInput* in : inputs) {
    Value t = Value::Object();
    t.Set("name", Value(in->Name()));
    Value shape = Value::Array();
    for (int64_t d : in->Shape()) shape.Append(Value(d));
    t.Set("shape", std::move(shape));
    t.Set("datatype", Value(in->Datatype()));
    if (in->IsSharedMemory()) {
      std::string region;
      size_t bs, off;
      in->SharedMemoryInfo(&region, &bs, &off);
      Value p = Value::Object();
      p.Set("shared_memory_region", Value(region));
      p.Set("shared_memory_byte_size", Value(static_cast<uint64_t>(bs)));
      if (off) p.Set("shared_memory_offset", Value(static_cast<uint64_t>(off)));
      t.Set("parameters", std::move(p));
    } else if (in->BinaryData()) {
      size_t bs;
      in->ByteSize(&bs);
      Value p = Value::Object();
      p.Set("binary_data_size", Value(static_cast<uint64_t>(bs)));
      t.Set("parameters", std::move(p));
    } else {
      Value data;
      Error e = InputToJson(in, &data);
      if (!e.IsOk()) return e;
      t.Set("data", std::move(data));
    }
    ins.Append(std::move(t));
  }
  req.Set("inputs", std::move(ins));
  if (!outputs.empty()) {
    Value outs = Value::Array();
    for (const InferRequestedOutput* o : outputs) {
      Value t = Value::Object();
      t.Set("name", Value(o->Name()));
      Value p = Value::Object();
      if (o->ClassificationCount() > 0) p.Set("classification", Value(static_cast<uint64_t>(o->ClassificationCount())));
      if (o->IsSharedMemory()) {
        std::string region;
        size_t bs, off;
        o->SharedMemoryInfo(&region, &bs, &off);
        p.Set("shared_memory_region", Value(region));
        p.Set("shared_memory_byte_size", Value(static_cast<uint64_t>(bs)));
        if (off) p.Set("shared_memory_offset", Value(static_cast<uint64_t>(off)));
      } else {
        p.Set("binary_data", Value(o->BinaryData()));
      }
      t.Set("parameters", std::move(p));
      outs.Append(std::move(t));
    }
    req.Set("outputs", std::move(outs));
  }
  req.Write(out);
  return Error::Success;
}

}  // namespace

//==============================================================================
// Blocking connection
//==============================================================================
class HttpConnection {
 public:
  Socket sock;
  HttpResponseParser parser;
  char rbuf[1 << 16];
};

struct HttpPreparedRequest {
  std::string head;                                      // request line + headers
  std::string json;                                      // JSON header (body part 0)
  std::string owned;                                     // compressed body if any
  std::vector<std::pair<const char*, size_t>> body;      // body parts (zero-copy)
  size_t body_len = 0;
  uint64_t timeout_us = 0;
  // async state
  InferenceServerClient::OnCompleteFn callback;
  RequestTimers timers;
  uint64_t deadline_ns = 0;
};

//==============================================================================
// Async engine: one epoll loop, non-blocking connections, one request each.
//==============================================================================
class HttpAsyncEngine {
 public:
  explicit HttpAsyncEngine(InferenceServerHttpClient* client) : client_(client)
  {
    ep_ = epoll_create1(EPOLL_CLOEXEC);
    ev_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    struct epoll_event e;
    e.events = EPOLLIN;
    e.data.ptr = nullptr;
    epoll_ctl(ep_, EPOLL_CTL_ADD, ev_, &e);
    worker_ = std::thread([this] { Loop(); });
  }
  ~HttpAsyncEngine()
  {
    {
      std::lock_guard<std::mutex> lk(mu_);
      exiting_ = true;
    }
    Wake();
    worker_.join();
    for (auto* c : idle_) delete c;
    close(ep_);
    close(ev_);
  }
  void Submit(std::unique_ptr<HttpPreparedRequest> r)
  {
    {
      std::lock_guard<std::mutex> lk(mu_);
      incoming_.push_back(std::move(r));
    }
    Wake();
  }

 private:
  struct Conn {
    Socket sock;
    HttpResponseParser parser;
    std::unique_ptr<HttpPreparedRequest> req;
    std::vector<struct iovec> iov;
    size_t iov_idx = 0;
  };

  void Wake()
  {
    uint64_t one = 1;
    ssize_t w = write(ev_, &one, sizeof(one));
    (void)w;
  }

  void Complete(Conn* c, const std::string& err)
  {
    std::unique_ptr<HttpPreparedRequest> req = std::move(c->req);
    req->timers.CaptureTimestamp(K::RECV_END);
    req->timers.CaptureTimestamp(K::REQUEST_END);
    if (c->parser.first_byte_ns()) req->timers.SetTimestamp(K::RECV_START, c->parser.first_byte_ns());
    else req->timers.SetTimestamp(K::RECV_START, req->timers.Timestamp(K::RECV_END));
    InferResult* result = nullptr;
    std::string body;
    size_t hl = 0;
    long code = err.empty() ? c->parser.status() : 0;
    if (err.empty()) {
      body.swap(c->parser.body());
      std::string enc = HeaderValue(c->parser.headers(), "content-encoding");
      if (enc == "gzip" || enc == "deflate") {
        std::string dec;
        if (Decompress(body, &dec)) body.swap(dec);
      }
      std::string h = HeaderValue(c->parser.headers(), kInferHeaderContentLengthHTTPHeader);
      if (!h.empty()) hl = std::strtoull(h.c_str(), nullptr, 10);
    }
    InferResultHttp::Create(&result, std::move(body), hl, code, err);
    if (err.empty()) client_->UpdateInferStat(req->timers);
    if (req->callback) req->callback(result);
    else delete result;
  }

  void Release(Conn* c, bool reuse)
  {
    epoll_ctl(ep_, EPOLL_CTL_DEL, c->sock.fd(), nullptr);
    active_.erase(c->sock.fd());
    if (reuse && c->parser.keep_alive() && idle_.size() < 1024) {
      idle_.push_back(c);
    } else {
      c->sock.Close();
      delete c;
    }
    --inflight_;
  }

  bool Start(std::unique_ptr<HttpPreparedRequest> r)
  {
    Conn* c = nullptr;
    while (!idle_.empty()) {
      c = idle_.back();
      idle_.pop_back();
      if (c->sock.IsOpen()) break;
      delete c;
      c = nullptr;
    }
    if (!c) {
      c = new Conn();
      TlsConfig tls;
      tls.enabled = client_->use_ssl_;
      tls.verify_peer = client_->ssl_options_.verify_peer != 0;
      tls.verify_host = client_->ssl_options_.verify_host != 0;
      tls.ca_info = client_->ssl_options_.ca_info;
      tls.cert = client_->ssl_options_.cert;
      tls.key = client_->ssl_options_.key;
      std::string err = c->sock.Connect(client_->host_, client_->port_, 10000000, tls);
      if (!err.empty()) {
        c->req = std::move(r);
        ++inflight_;
        Complete(c, err);
        --inflight_;
        delete c;
        return false;
      }
      c->sock.SetNonBlocking(true);
    }
    c->req = std::move(r);
    c->parser.Reset();
    c->iov.clear();
    c->iov.push_back({const_cast<char*>(c->req->head.data()), c->req->head.size()});
    for (const auto& p : c->req->body) c->iov.push_back({const_cast<char*>(p.first), p.second});
    c->iov_idx = 0;
    c->req->timers.CaptureTimestamp(K::SEND_START);
    ++inflight_;
    active_[c->sock.fd()] = c;
    struct epoll_event e;
    e.events = EPOLLOUT | EPOLLIN;
    e.data.ptr = c;
    epoll_ctl(ep_, EPOLL_CTL_ADD, c->sock.fd(), &e);
    OnWritable(c);
    return true;
  }

  void OnWritable(Conn* c)
  {
    while (c->iov_idx < c->iov.size()) {
      ssize_t n = c->sock.Writev(&c->iov[c->iov_idx], static_cast<int>(c->iov.size() - c->iov_idx));
      if (n < 0) {
        Complete(c, "failed to send request: connection error");
        Release(c, false);
        return;
      }
      if (n == 0) return;  // would block
      size_t left = static_cast<size_t>(n);
      while (left && c->iov_idx < c->iov.size()) {
        auto& v = c->iov[c->iov_idx];
        if (left >= v.iov_len) {
          left -= v.iov_len;
          ++c->iov_idx;
        } else {
          v.iov_base = static_cast<char*>(v.iov_base) + left;
          v.iov_len -= left;
          left = 0;
        }
      }
    }
    c->req->timers.CaptureTimestamp(K::SEND_END);
    struct epoll_event e;
    e.events = EPOLLIN;
    e.data.ptr = c;
    epoll_ctl(ep_, EPOLL_CTL_MOD, c->sock.fd(), &e);
  }

  void OnReadable(Conn* c)
  {
    char buf[1 << 16];
    while (true) {
      ssize_t n = c->sock.Read(buf, sizeof(buf));
      if (n == -2) return;
      if (n <= 0) {
        if (c->parser.state() == HttpResponseParser::State::Body && !c->parser.keep_alive() && n == 0) {
          Complete(c, "");
          Release(c, false);
        } else {
          Complete(c, "connection closed by server");
          Release(c, false);
        }
        return;
      }
      c->parser.Feed(buf, static_cast<size_t>(n));
      if (c->parser.state() == HttpResponseParser::State::Error) {
        Complete(c, "malformed HTTP response: " + c->parser.error());
        Release(c, false);
        return;
      }
      if (c->parser.state() == HttpResponseParser::State::Done) {
        Complete(c, "");
        Release(c, true);
        return;
      }
    }
  }

  void Loop()
  {
    std::vector<struct epoll_event> events(256);
    while (true) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        if (exiting_ && incoming_.empty() && waiting_.empty() && inflight_ == 0) break;
        while (!incoming_.empty()) {
          waiting_.push_back(std::move(incoming_.front()));
          incoming_.pop_front();
        }
      }
      while (!waiting_.empty() && inflight_ < client_->max_async_conns_) {
        auto r = std::move(waiting_.front());
        waiting_.pop_front();
        Start(std::move(r));
      }
      // timeout = nearest deadline
      uint64_t now = RequestTimers::Now();
      int timeout_ms = 100;
      for (auto& kv : active_) {
        uint64_t d = kv.second->req ? kv.second->req->deadline_ns : 0;
        if (d) timeout_ms = std::min<int64_t>(timeout_ms, d > now ? static_cast<int64_t>((d - now) / 1000000) + 1 : 0);
      }
      int n = epoll_wait(ep_, events.data(), static_cast<int>(events.size()), timeout_ms);
      for (int i = 0; i < n; ++i) {
        if (events[i].data.ptr == nullptr) {
          uint64_t v;
          ssize_t r = read(ev_, &v, sizeof(v));
          (void)r;
          continue;
        }
        Conn* c = static_cast<Conn*>(events[i].data.ptr);
        if (active_.find(c->sock.fd()) == active_.end() || active_[c->sock.fd()] != c) continue;
        if (events[i].events & (EPOLLERR | EPOLLHUP)) {
          if (events[i].events & EPOLLIN) {
            OnReadable(c);
          } else {
            Complete(c, "connection error");
            Release(c, false);
          }
          continue;
        }
        if (events[i].events & EPOLLOUT) OnWritable(c);
        if ((events[i].events & EPOLLIN) && active_.count(c->sock.fd())) OnReadable(c);
      }
      // deadlines
      now = RequestTimers::Now();
      std::vector<Conn*> expired;
      for (auto& kv : active_)
        if (kv.second->req && kv.second->req->deadline_ns && kv.second->req->deadline_ns <= now)
          expired.push_back(kv.second);
      for (Conn* c : expired) {
        Complete(c, "Deadline Exceeded");
        Release(c, false);
      }
    }
  }

  InferenceServerHttpClient* client_;
  int ep_, ev_;
  std::thread worker_;
  std::mutex mu_;
  bool exiting_ = false;
  std::deque<std::unique_ptr<HttpPreparedRequest>> incoming_;
  std::deque<std::unique_ptr<HttpPreparedRequest>> waiting_;
  std::unordered_map<int, Conn*> active_;
  std::vector<Conn*> idle_;
  size_t inflight_ = 0;
};

//==============================================================================
// Client
//==============================================================================
Error
InferenceServerHttpClient::Create(
    std::unique_ptr<InferenceServerHttpClient>* client, const std::string& server_url, bool verbose,
    const HttpSslOptions& ssl_options)
{
  client->reset(new InferenceServerHttpClient(server_url, verbose, ssl_options));
  return Error::Success;
}

InferenceServerHttpClient::InferenceServerHttpClient(const std::string& url, bool verbose, const HttpSslOptions& ssl_options)
    : InferenceServerClient(verbose), port_(80), use_ssl_(false), ssl_options_(ssl_options)
{
  std::string u = url;
  if (u.compare(0, 8, "https://") == 0) {
    use_ssl_ = true;
    u = u.substr(8);
  } else if (u.compare(0, 7, "http://") == 0) {
    u = u.substr(7);
  }
  size_t slash = u.find('/');
  std::string hostport = u.substr(0, slash);
  if (slash != std::string::npos) {
    base_path_ = u.substr(slash);
    while (!base_path_.empty() && base_path_.back() == '/') base_path_.pop_back();
  }
  // host:port, [v6]:port, or host (default port)
  size_t colon = hostport.rfind(':');
  size_t bracket = hostport.find(']');
  bool has_port = colon != std::string::npos && (bracket == std::string::npos || colon > bracket);
  host_ = has_port ? hostport.substr(0, colon) : hostport;
  port_ = has_port ? std::atoi(hostport.c_str() + colon + 1) : (use_ssl_ ? 443 : 80);
  if (!host_.empty() && host_.front() == '[') host_ = host_.substr(1, host_.size() - 2);
  sync_conn_.reset(new HttpConnection());
}

InferenceServerHttpClient::~InferenceServerHttpClient()
{
  engine_.reset();
}

Error
InferenceServerHttpClient::Request(
    const std::string& method, std::string& uri, const std::vector<std::pair<const char*, size_t>>& body,
    const Headers& headers, const Parameters& query_params, long* http_code, std::string* response_body,
    std::map<std::string, std::string>* response_headers, uint64_t timeout_us, RequestTimers* timers)
{
  std::string full = base_path_ + "/" + uri + QueryString(query_params);
  size_t total = 0;
  for (const auto& p : body) total += p.second;
  std::string head = method + " " + full + " HTTP/1.1\r\n";
  AppendHeaderLine(&head, "Host", host_ + ":" + std::to_string(port_));
  for (const auto& kv : headers) AppendHeaderLine(&head, kv.first, kv.second);
  if (method != "GET" || total) AppendHeaderLine(&head, "Content-Length", std::to_string(total));
  head.append("\r\n");
  if (verbose_) std::cout << method << " " << full << std::endl;

  std::lock_guard<std::mutex> lk(sync_mu_);
  HttpConnection* c = sync_conn_.get();
  for (int attempt = 0; attempt < 2; ++attempt) {
    bool reused = c->sock.IsOpen();
    if (!reused) {
      TlsConfig tls;
      tls.enabled = use_ssl_;
      tls.verify_peer = ssl_options_.verify_peer != 0;
      tls.verify_host = ssl_options_.verify_host != 0;
      tls.ca_info = ssl_options_.ca_info;
      tls.cert = ssl_options_.cert;
      tls.key = ssl_options_.key;
      tls.cert_der = ssl_options_.cert_type == HttpSslOptions::CERT_DER;
      tls.key_der = ssl_options_.key_type == HttpSslOptions::KEY_DER;
      std::string err = c->sock.Connect(host_, port_, timeout_us ? timeout_us : 60000000, tls);
      if (!err.empty()) return Error(err);
    }
    std::vector<struct iovec> iov;
    iov.push_back({const_cast<char*>(head.data()), head.size()});
    for (const auto& p : body) iov.push_back({const_cast<char*>(p.first), p.second});
    if (timers) timers->CaptureTimestamp(K::SEND_START);
    size_t idx = 0;
    bool send_failed = false;
    const uint64_t t0 = RequestTimers::Now();
    while (idx < iov.size()) {
      ssize_t n = c->sock.Writev(&iov[idx], static_cast<int>(iov.size() - idx));
      if (n < 0) {
        send_failed = true;
        break;
      }
      size_t left = static_cast<size_t>(n);
      while (left && idx < iov.size()) {
        if (left >= iov[idx].iov_len) {
          left -= iov[idx].iov_len;
          ++idx;
        } else {
          iov[idx].iov_base = static_cast<char*>(iov[idx].iov_base) + left;
          iov[idx].iov_len -= left;
          left = 0;
        }
      }
      if (n == 0) c->sock.Wait(true, 1000000);
    }
    if (timers) timers->CaptureTimestamp(K::SEND_END);
    if (send_failed) {
      c->sock.Close();
      if (reused && attempt == 0) continue;
      return Error("failed to send HTTP request");
    }
    c->parser.Reset(method == "HEAD");
    bool retry = false;
    while (c->parser.state() != HttpResponseParser::State::Done) {
      if (timeout_us) {
        uint64_t el = (RequestTimers::Now() - t0) / 1000;
        if (el >= timeout_us || !c->sock.Wait(false, static_cast<int64_t>(timeout_us - el))) {
          c->sock.Close();
          return Error("Deadline Exceeded");
        }
      }
      ssize_t n = c->sock.Read(c->rbuf, sizeof(c->rbuf));
      if (n == -2) continue;
      if (n <= 0) {
        if (c->parser.state() == HttpResponseParser::State::Body && !c->parser.keep_alive() && n == 0) break;
        c->sock.Close();
        if (reused && attempt == 0 && c->parser.state() == HttpResponseParser::State::Headers) {
          retry = true;
          break;
        }
        return Error("connection closed by server");
      }
      c->parser.Feed(c->rbuf, static_cast<size_t>(n));
      if (c->parser.state() == HttpResponseParser::State::Error) {
        c->sock.Close();
        return Error("malformed HTTP response: " + c->parser.error());
      }
    }
    if (retry) continue;
    if (timers) {
      timers->SetTimestamp(K::RECV_START, c->parser.first_byte_ns() ? c->parser.first_byte_ns() : RequestTimers::Now());
      timers->CaptureTimestamp(K::RECV_END);
    }
    if (http_code) *http_code = c->parser.status();
    if (response_headers) *response_headers = c->parser.headers();
    if (response_body) response_body->swap(c->parser.body());
    if (!c->parser.keep_alive()) c->sock.Close();
    if (verbose_ && response_body) std::cout << *response_body << std::endl;
    return Error::Success;
  }
  return Error("failed to send HTTP request");
}

Error
InferenceServerHttpClient::Get(
    std::string& request_uri, const Headers& headers, const Parameters& query_params, std::string* response,
    long* http_code)
{
  long code = 0;
  std::string body;
  Error e = Request("GET", request_uri, {}, headers, query_params, &code, &body, nullptr, 0);
  if (!e.IsOk()) return e;
  if (http_code) *http_code = code;
  if (code != 200 && http_code == nullptr) {
    Value v;
    std::string err;
    if (json::Parse(body, &v, &err) && v.IsObject() && v.Find("error")) return Error(v.Find("error")->AsString());
    return Error("HTTP " + std::to_string(code));
  }
  if (response) response->swap(body);
  return Error::Success;
}

Error
InferenceServerHttpClient::Post(
    std::string& request_uri, const std::string& request, const Headers& headers, const Parameters& query_params,
    std::string* response, long* http_code)
{
  long code = 0;
  std::string body;
  std::vector<std::pair<const char*, size_t>> parts;
  if (!request.empty()) parts.push_back({request.data(), request.size()});
  Error e = Request("POST", request_uri, parts, headers, query_params, &code, &body, nullptr, 0);
  if (!e.IsOk()) return e;
  if (http_code) *http_code = code;
  if (code != 200) {
    Value v;
    std::string err;
    if (json::Parse(body, &v, &err) && v.IsObject() && v.Find("error")) return Error(v.Find("error")->AsString());
    return Error("HTTP " + std::to_string(code));
  }
  if (response) response->swap(body);
  return Error::Success;
}

static std::string
ModelUri(const std::string& model, const std::string& version, const std::string& suffix = "")
{
  std::string u = "v2/models/" + UrlEncode(model);
  if (!version.empty()) u += "/versions/" + version;
  return u + suffix;
}

Error
InferenceServerHttpClient::IsServerLive(bool* live, const Headers& headers, const Parameters& query_params)
{
  std::string uri = "v2/health/live";
  long code = 0;
  Error e = Get(uri, headers, query_params, nullptr, &code);
  *live = e.IsOk() && code == 200;
  return e;
}

Error
InferenceServerHttpClient::IsServerReady(bool* ready, const Headers& headers, const Parameters& query_params)
{
  std::string uri = "v2/health/ready";
  long code = 0;
  Error e = Get(uri, headers, query_params, nullptr, &code);
  *ready = e.IsOk() && code == 200;
  return e;
}

Error
InferenceServerHttpClient::IsModelReady(
    bool* ready, const std::string& model_name, const std::string& model_version, const Headers& headers,
    const Parameters& query_params)
{
  std::string uri = ModelUri(model_name, model_version, "/ready");
  long code = 0;
  Error e = Get(uri, headers, query_params, nullptr, &code);
  *ready = e.IsOk() && code == 200;
  return e;
}

Error
InferenceServerHttpClient::ServerMetadata(std::string* server_metadata, const Headers& headers, const Parameters& q)
{
  std::string uri = "v2";
  return Get(uri, headers, q, server_metadata);
}

Error
InferenceServerHttpClient::ModelMetadata(
    std::string* model_metadata, const std::string& model_name, const std::string& model_version,
    const Headers& headers, const Parameters& q)
{
  std::string uri = ModelUri(model_name, model_version);
  return Get(uri, headers, q, model_metadata);
}

Error
InferenceServerHttpClient::ModelConfig(
    std::string* model_config, const std::string& model_name, const std::string& model_version,
    const Headers& headers, const Parameters& q)
{
  std::string uri = ModelUri(model_name, model_version, "/config");
  return Get(uri, headers, q, model_config);
}

Error
InferenceServerHttpClient::ModelRepositoryIndex(std::string* repository_index, const Headers& headers, const Parameters& q)
{
  std::string uri = "v2/repository/index";
  return Post(uri, "", headers, q, repository_index);
}

Error
InferenceServerHttpClient::LoadModel(
    const std::string& model_name, const Headers& headers, const Parameters& q, const std::string& config,
    const std::map<std::string, std::vector<char>>& files)
{
  std::string uri = "v2/repository/models/" + UrlEncode(model_name) + "/load";
  Value req = Value::Object();
  if (!config.empty() || !files.empty()) {
    Value p = Value::Object();
    if (!config.empty()) p.Set("config", Value(config));
    for (const auto& kv : files) p.Set(kv.first, Value(Base64EncodeLibb64(kv.second.data(), kv.second.size())));
    req.Set("parameters", std::move(p));
  }
  return Post(uri, req.Serialize(), headers, q, nullptr);
}

Error
InferenceServerHttpClient::UnloadModel(const std::string& model_name, const Headers& headers, const Parameters& q)
{
  std::string uri = "v2/repository/models/" + UrlEncode(model_name) + "/unload";
  return Post(uri, "", headers, q, nullptr);
}

Error
InferenceServerHttpClient::ModelInferenceStatistics(
    std::string* infer_stat, const std::string& model_name, const std::string& model_version, const Headers& headers,
    const Parameters& q)
{
  std::string uri = model_name.empty() ? std::string("v2/models/stats") : ModelUri(model_name, model_version, "/stats");
  return Get(uri, headers, q, infer_stat);
}

Error
InferenceServerHttpClient::UpdateTraceSettings(
    std::string* response, const std::string& model_name,
    const std::map<std::string, std::vector<std::string>>& settings, const Headers& headers, const Parameters& q)
{
  std::string uri = model_name.empty() ? std::string("v2/trace/setting")
                                       : "v2/models/" + UrlEncode(model_name) + "/trace/setting";
  Value req = Value::Object();
  for (const auto& kv : settings) {
    if (kv.second.empty()) {
      req.Set(kv.first, Value());  // null clears the setting
    } else if (kv.first == "trace_level") {
      Value a = Value::Array();
      for (const auto& s : kv.second) a.Append(Value(s));
      req.Set(kv.first, std::move(a));
    } else {
      req.Set(kv.first, Value(kv.second[0]));
    }
  }
  return Post(uri, req.Serialize(), headers, q, response);
}

Error
InferenceServerHttpClient::GetTraceSettings(
    std::string* settings, const std::string& model_name, const Headers& headers, const Parameters& q)
{
  std::string uri = model_name.empty() ? std::string("v2/trace/setting")
                                       : "v2/models/" + UrlEncode(model_name) + "/trace/setting";
  return Get(uri, headers, q, settings);
}

Error
InferenceServerHttpClient::UpdateLogSettings(
    std::string* response, const std::map<std::string, std::string>& settings, const Headers& headers,
    const Parameters& q)
{
  std::string uri = "v2/logging";
  Value req = Value::Object();
  for (const auto& kv : settings) {
    if (kv.first == "log_file" || kv.first == "log_format") req.Set(kv.first, Value(kv.second));
    else if (kv.first == "log_verbose_level") req.Set(kv.first, Value(static_cast<int64_t>(std::stoll(kv.second))));
    else req.Set(kv.first, Value(kv.second == "true" || kv.second == "1"));
  }
  return Post(uri, req.Serialize(), headers, q, response);
}

Error
InferenceServerHttpClient::GetLogSettings(std::string* settings, const Headers& headers, const Parameters& q)
{
  std::string uri = "v2/logging";
  return Get(uri, headers, q, settings);
}

Error
InferenceServerHttpClient::SystemSharedMemoryStatus(
    std::string* status, const std::string& region_name, const Headers& headers, const Parameters& q)
{
  std::string uri = region_name.empty() ? std::string("v2/systemsharedmemory/status")
                                        : "v2/systemsharedmemory/region/" + UrlEncode(region_name) + "/status";
  return Get(uri, headers, q, status);
}

Error
InferenceServerHttpClient::RegisterSystemSharedMemory(
    const std::string& name, const std::string& key, const size_t byte_size, const size_t offset,
    const Headers& headers, const Parameters& q)
{
  std::string uri = "v2/systemsharedmemory/region/" + UrlEncode(name) + "/register";
  Value req = Value::Object();
  req.Set("key", Value(key));
  req.Set("offset", Value(static_cast<uint64_t>(offset)));
  req.Set("byte_size", Value(static_cast<uint64_t>(byte_size)));
  return Post(uri, req.Serialize(), headers, q, nullptr);
}

Error
InferenceServerHttpClient::UnregisterSystemSharedMemory(const std::string& name, const Headers& headers, const Parameters& q)
{
  std::string uri = name.empty() ? std::string("v2/systemsharedmemory/unregister")
                                 : "v2/systemsharedmemory/region/" + UrlEncode(name) + "/unregister";
  return Post(uri, "", headers, q, nullptr);
}

Error
InferenceServerHttpClient::CudaSharedMemoryStatus(
    std::string* status, const std::string& region_name, const Headers& headers, const Parameters& q)
{
  std::string uri = region_name.empty() ? std::string("v2/cudasharedmemory/status")
                                        : "v2/cudasharedmemory/region/" + UrlEncode(region_name) + "/status";
  return Get(uri, headers, q, status);
}

Error
InferenceServerHttpClient::RegisterCudaSharedMemory(
    const std::string& name, const cudaIpcMemHandle_t& cuda_shm_handle, const size_t device_id,
    const size_t byte_size, const Headers& headers, const Parameters& q)
{
  std::string uri = "v2/cudasharedmemory/region/" + UrlEncode(name) + "/register";
  Value req = Value::Object();
  Value h = Value::Object();
  h.Set("b64", Value(Base64EncodeLibb64(&cuda_shm_handle, sizeof(cuda_shm_handle))));
  req.Set("raw_handle", std::move(h));
  req.Set("device_id", Value(static_cast<uint64_t>(device_id)));
  req.Set("byte_size", Value(static_cast<uint64_t>(byte_size)));
  return Post(uri, req.Serialize(), headers, q, nullptr);
}

Error
InferenceServerHttpClient::UnregisterCudaSharedMemory(const std::string& name, const Headers& headers, const Parameters& q)
{
  std::string uri = name.empty() ? std::string("v2/cudasharedmemory/unregister")
                                 : "v2/cudasharedmemory/region/" + UrlEncode(name) + "/unregister";
  return Post(uri, "", headers, q, nullptr);
}

//==============================================================================
Error
InferenceServerHttpClient::GenerateRequestBody(
    std::vector<char>* request_body, size_t* header_length, const InferOptions& options,
    const std::vector<InferInput*>& inputs, const std::vector<const InferRequestedOutput*>& outputs)
{
  std::string js;
  Error e = BuildRequestJson(options, inputs, outputs, &js);
  if (!e.IsOk()) return e;
  request_body->assign(js.begin(), js.end());
  *header_length = js.size();
  for (InferInput* in : inputs) {
    if (in->IsSharedMemory() || !in->BinaryData()) continue;
    for (size_t i = 0; i < in->Buffers().size(); ++i) {
      const char* p = reinterpret_cast<const char*>(in->Buffers()[i]);
      request_body->insert(request_body->end(), p, p + in->BufferSizes()[i]);
    }
  }
  return Error::Success;
}

Error
InferenceServerHttpClient::ParseResponseBody(
    InferResult** result, const std::vector<char>& response_body, const size_t header_length)
{
  std::string body(response_body.begin(), response_body.end());
  return InferResultHttp::Create(result, std::move(body), header_length, 200, "");
}

Error
InferenceServerHttpClient::PrepareInfer(
    const InferOptions& options, const std::vector<InferInput*>& inputs,
    const std::vector<const InferRequestedOutput*>& outputs, const Headers& headers, const Parameters& query_params,
    CompressionType request_compression, CompressionType response_compression, HttpPreparedRequest* req)
{
  Error e = BuildRequestJson(options, inputs, outputs, &req->json);
  if (!e.IsOk()) return e;
  req->body.clear();
  req->body.push_back({req->json.data(), req->json.size()});
  bool any_binary = false;
  for (InferInput* in : inputs) {
    if (in->IsSharedMemory() || !in->BinaryData()) continue;
    in->PrepareForRequest();
    for (size_t i = 0; i < in->Buffers().size(); ++i) {
      req->body.push_back({reinterpret_cast<const char*>(in->Buffers()[i]), in->BufferSizes()[i]});
      any_binary = true;
    }
  }
  std::string uri = base_path_ + "/" + ModelUri(options.model_name_, options.model_version_, "/infer") +
                    QueryString(query_params);
  std::string extra;
  if (request_compression != CompressionType::NONE) {
    bool gz = request_compression == CompressionType::GZIP;
    if (!Compress(req->body, gz, &req->owned)) return Error("failed to compress request body");
    req->body.clear();
    req->body.push_back({req->owned.data(), req->owned.size()});
    AppendHeaderLine(&extra, "Content-Encoding", gz ? "gzip" : "deflate");
  }
  if (response_compression == CompressionType::GZIP) AppendHeaderLine(&extra, "Accept-Encoding", "gzip");
  else if (response_compression == CompressionType::DEFLATE) AppendHeaderLine(&extra, "Accept-Encoding", "deflate");
  req->body_len = 0;
  for (const auto& p : req->body) req->body_len += p.second;
  req->head = "POST " + uri + " HTTP/1.1\r\n";
  AppendHeaderLine(&req->head, "Host", host_ + ":" + std::to_string(port_));
  AppendHeaderLine(&req->head, "Content-Type", any_binary ? "application/octet-stream" : "application/json");
  AppendHeaderLine(&req->head, kInferHeaderContentLengthHTTPHeader, std::to_string(req->json.size()));
  for (const auto& kv : headers) AppendHeaderLine(&req->head, kv.first, kv.second);
  req->head.append(extra);
  AppendHeaderLine(&req->head, "Content-Length", std::to_string(req->body_len));
  req->head.append("\r\n");
  req->timeout_us = options.client_timeout_;
  return Error::Success;
}

Error
InferenceServerHttpClient::Infer(
    InferResult** result, const InferOptions& options, const std::vector<InferInput*>& inputs,
    const std::vector<const InferRequestedOutput*>& outputs, const Headers& headers, const Parameters& query_params,
    const CompressionType request_compression_algorithm, const CompressionType response_compression_algorithm)
{
  trace::Range range("tc.http.Infer");
  RequestTimers timers;
  timers.CaptureTimestamp(K::REQUEST_START);
  HttpPreparedRequest req;
  Error e = PrepareInfer(options, inputs, outputs, headers, query_params, request_compression_algorithm,
                         response_compression_algorithm, &req);
  if (!e.IsOk()) return e;
  // the prepared head already carries every header: send it verbatim
  std::lock_guard<std::mutex> lk(sync_mu_);
  HttpConnection* c = sync_conn_.get();
  std::string err;
  long code = 0;
  std::string body;
  std::map<std::string, std::string> rh;
  for (int attempt = 0; attempt < 2; ++attempt) {
    bool reused = c->sock.IsOpen();
    if (!reused) {
      TlsConfig tls;
      tls.enabled = use_ssl_;
      tls.verify_peer = ssl_options_.verify_peer != 0;
      tls.verify_host = ssl_options_.verify_host != 0;
      tls.ca_info = ssl_options_.ca_info;
      tls.cert = ssl_options_.cert;
      tls.key = ssl_options_.key;
      err = c->sock.Connect(host_, port_, 60000000, tls);
      if (!err.empty()) return Error(err);
    }
    std::vector<struct iovec> iov;
    iov.push_back({const_cast<char*>(req.head.data()), req.head.size()});
    for (const auto& p : req.body) iov.push_back({const_cast<char*>(p.first), p.second});
    timers.CaptureTimestamp(K::SEND_START);
    size_t idx = 0;
    bool failed = false;
    const uint64_t t0 = RequestTimers::Now();
    while (idx < iov.size()) {
      ssize_t n = c->sock.Writev(&iov[idx], static_cast<int>(iov.size() - idx));
      if (n < 0) {
        failed = true;
        break;
      }
      size_t left = static_cast<size_t>(n);
      while (left && idx < iov.size()) {
        if (left >= iov[idx].iov_len) {
          left -= iov[idx].iov_len;
          ++idx;
        } else {
          iov[idx].iov_base = static_cast<char*>(iov[idx].iov_base) + left;
          iov[idx].iov_len -= left;
          left = 0;
        }
      }
    }
    timers.CaptureTimestamp(K::SEND_END);
    if (failed) {
      c->sock.Close();
      if (reused && attempt == 0) continue;
      return Error("failed to send inference request");
    }
    c->parser.Reset();
    bool retry = false;
    err.clear();
    while (c->parser.state() != HttpResponseParser::State::Done) {
      if (req.timeout_us) {
        uint64_t el = (RequestTimers::Now() - t0) / 1000;
        if (el >= req.timeout_us || !c->sock.Wait(false, static_cast<int64_t>(req.timeout_us - el))) {
          c->sock.Close();
          err = "Deadline Exceeded";
          break;
        }
      }
      ssize_t n = c->sock.Read(c->rbuf, sizeof(c->rbuf));
      if (n == -2) continue;
      if (n <= 0) {
        if (c->parser.state() == HttpResponseParser::State::Body && !c->parser.keep_alive() && n == 0) break;
        c->sock.Close();
        if (reused && attempt == 0 && c->parser.state() == HttpResponseParser::State::Headers) {
          retry = true;
          break;
        }
        err = "connection closed by server";
        break;
      }
      c->parser.Feed(c->rbuf, static_cast<size_t>(n));
      if (c->parser.state() == HttpResponseParser::State::Error) {
        c->sock.Close();
        err = "malformed HTTP response: " + c->parser.error();
        break;
      }
    }
    if (retry) continue;
    break;
  }
  timers.SetTimestamp(K::RECV_START, c->parser.first_byte_ns() ? c->parser.first_byte_ns() : RequestTimers::Now());
  timers.CaptureTimestamp(K::RECV_END);
  timers.CaptureTimestamp(K::REQUEST_END);
  size_t hl = 0;
  if (err.empty()) {
    code = c->parser.status();
    body.swap(c->parser.body());
    rh = c->parser.headers();
    if (!c->parser.keep_alive()) c->sock.Close();
    std::string enc = HeaderValue(rh, "content-encoding");
    if (enc == "gzip" || enc == "deflate") {
      std::string dec;
      if (Decompress(body, &dec)) body.swap(dec);
    }
    std::string h = HeaderValue(rh, kInferHeaderContentLengthHTTPHeader);
    if (!h.empty()) hl = std::strtoull(h.c_str(), nullptr, 10);
  }
  InferResultHttp::Create(result, std::move(body), hl, code, err);
  if (err.empty()) UpdateInferStat(timers);
  if (verbose_) std::cout << (*result)->DebugString() << std::endl;
  return (*result)->RequestStatus();
}

Error
InferenceServerHttpClient::AsyncInfer(
    OnCompleteFn callback, const InferOptions& options, const std::vector<InferInput*>& inputs,
    const std::vector<const InferRequestedOutput*>& outputs, const Headers& headers, const Parameters& query_params,
    const CompressionType request_compression_algorithm, const CompressionType response_compression_algorithm)
{
  if (callback == nullptr) {
    return Error("Callback function must be provided along with AsyncInfer() call.");
  }
  auto req = std::make_unique<HttpPreparedRequest>();
  req->timers.CaptureTimestamp(K::REQUEST_START);
  Error e = PrepareInfer(options, inputs, outputs, headers, query_params, request_compression_algorithm,
                         response_compression_algorithm, req.get());
  if (!e.IsOk()) return e;
  req->callback = callback;
  if (options.client_timeout_) req->deadline_ns = RequestTimers::Now() + options.client_timeout_ * 1000;
  {
    std::lock_guard<std::mutex> lk(mutex_);
    if (!engine_) engine_.reset(new HttpAsyncEngine(this));
  }
  engine_->Submit(std::move(req));
  return Error::Success;
}

Error
InferenceServerHttpClient::InferMulti(
    std::vector<InferResult*>* results, const std::vector<InferOptions>& options,
    const std::vector<std::vector<InferInput*>>& inputs,
    const std::vector<std::vector<const InferRequestedOutput*>>& outputs, const Headers& headers,
    const Parameters& query_params, const CompressionType req_c, const CompressionType resp_c)
{
  if (options.size() != 1 && options.size() != inputs.size()) {
    return Error("'options' must either contain 1 element or match size of 'inputs'");
  }
  if (outputs.size() > 1 && outputs.size() != inputs.size()) {
    return Error("'outputs' must either contain 0/1 element or match size of 'inputs'");
  }
  results->clear();
  Error first;
  for (size_t i = 0; i < inputs.size(); ++i) {
    const InferOptions& o = options.size() == 1 ? options[0] : options[i];
    static const std::vector<const InferRequestedOutput*> none;
    const auto& outs = outputs.empty() ? none : (outputs.size() == 1 ? outputs[0] : outputs[i]);
    InferResult* r = nullptr;
    Error e = Infer(&r, o, inputs[i], outs, headers, query_params, req_c, resp_c);
    if (!e.IsOk() && first.IsOk()) first = e;
    results->push_back(r);
  }
  return first;
}

Error
InferenceServerHttpClient::AsyncInferMulti(
    OnMultiCompleteFn callback, const std::vector<InferOptions>& options,
    const std::vector<std::vector<InferInput*>>& inputs,
    const std::vector<std::vector<const InferRequestedOutput*>>& outputs, const Headers& headers,
    const Parameters& query_params, const CompressionType req_c, const CompressionType resp_c)
{
  if (callback == nullptr) {
    return Error("Callback function must be provided along with AsyncInferMulti() call.");
  }
  if (options.size() != 1 && options.size() != inputs.size()) {
    return Error("'options' must either contain 1 element or match size of 'inputs'");
  }
  if (outputs.size() > 1 && outputs.size() != inputs.size()) {
    return Error("'outputs' must either contain 0/1 element or match size of 'inputs'");
  }
  struct Fanin {
    std::atomic<size_t> left;
    std::vector<InferResult*> results;
    OnMultiCompleteFn cb;
  };
  auto st = std::make_shared<Fanin>();
  st->left = inputs.size();
  st->results.resize(inputs.size(), nullptr);
  st->cb = callback;
  for (size_t i = 0; i < inputs.size(); ++i) {
    const InferOptions& o = options.size() == 1 ? options[0] : options[i];
    static const std::vector<const InferRequestedOutput*> none;
    const auto& outs = outputs.empty() ? none : (outputs.size() == 1 ? outputs[0] : outputs[i]);
    Error e = AsyncInfer(
        [st, i](InferResult* r) {
          st->results[i] = r;
          if (--st->left == 0) st->cb(st->results);
        },
        o, inputs[i], outs, headers, query_params, req_c, resp_c);
    if (!e.IsOk()) return e;
  }
  return Error::Success;
}

}}  // namespace triton::client

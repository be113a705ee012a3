// tcserve implementation: HTTP/2 server transport, proxy to the Python
// grpc.aio server, native ModelInfer fast path with a dynamic batcher.
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <nghttp2/nghttp2.h>
#include <pthread.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <queue>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "grpc_service.pb.h"
#include "h2.h"
#include "json.h"
#include "net.h"
#include "tcserve.h"
#include "batch_policy.h"
#include "trace.h"

namespace tcserve {

namespace tc = triton::client;

static uint64_t NowNs()
{
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

static const char kInferPath[] = "/inference.GRPCInferenceService/ModelInfer";

// gRPC status codes used here
enum { kOk = 0, kInvalidArgument = 3, kNotFound = 5, kInternal = 13, kUnavailable = 14 };

class Server;
class Loop;

// ---------------------------------------------------------------------------
struct Stream {
  int32_t id = 0;
  std::string path;
  std::vector<std::pair<std::string, std::string>> meta;
  std::string inbuf;
  bool end_stream = false;
  bool started = false;        // dispatched (unary) / upstream opened (streaming)
  bool streaming_rpc = false;
  // response
  bool response_submitted = false;
  std::deque<std::string> out;  // framed messages
  size_t out_pos = 0;
  bool finish = false;          // send trailers once `out` drains
  int status = 0;
  std::string message;
  bool trailers_sent = false;
  bool deferred = false;
  std::shared_ptr<tc::H2Call> upstream;
};

struct Conn {
  uint64_t id = 0;
  int fd = -1;
  Loop* loop = nullptr;
  nghttp2_session* s = nullptr;  // gRPC (h2c) connections
  // HTTP/1.1 (KServe REST) connections: requests parsed from `hin`, answered
  // strictly in request order (pipelining) through `ready`
  bool http1 = false;
  std::string hin;
  uint64_t req_seq = 0, resp_seq = 0;
  std::map<uint64_t, std::string> ready;
  bool close_after = false;
  std::unordered_map<int32_t, std::unique_ptr<Stream>> streams;
  std::string sendbuf;
  size_t sendpos = 0;
  bool closing = false;
  bool want_write = false;
};

// ---------------------------------------------------------------------------
// Native models
// ---------------------------------------------------------------------------
struct TensorDef {
  std::string name, dtype;
  std::vector<int64_t> dims;
  size_t sample_bytes = 0;
};

struct PendingReq {
  uint64_t conn_id;
  Loop* loop;
  int32_t stream_id;
  bool http = false;      // KServe REST request: reply as JSON header + binary outputs
  uint64_t http_seq = 0;  // position in its connection's request order
  bool http_close = false;
  int http_resp_enc = 0;  // response Content-Encoding: 0 none, 1 gzip, 2 deflate (zlib)
  std::string id;
  int32_t rows;
  std::vector<tcserve_ref> in;    // [n_inputs]
  std::vector<tcserve_ref> out;   // [n_outputs] (ptr 0: not requested / host)
  std::vector<bool> out_requested;
  std::vector<bool> out_shm;
  std::vector<std::string> out_region;
  std::vector<int64_t> out_region_bytes, out_region_offset;
  std::vector<std::string> host_out;  // host output buffers (non-shm)
  std::string body;                   // request message; raw inputs point into it
  std::vector<std::pair<int, size_t>> host_in_off;  // (input index, offset of its bytes in body)
  std::vector<std::shared_ptr<int>> pins;            // shm regions this request reads/writes
  uint64_t t_arrive = 0;
};

struct Stat {
  uint64_t count = 0, ns = 0;
};

struct BatchStat {
  uint64_t count = 0, in_ns = 0, infer_ns = 0, out_ns = 0;
};

struct NativeModel {
  std::string name, version;
  int max_batch = 0;
  uint64_t delay_ns = 0;
  std::vector<int> preferred;  // ascending; dynamic_batching.preferred_batch_size
  bool idle_dispatch = true;   // no queue delay while every instance is idle
  bool pipelined = false;      // a free instance takes the queue once it holds the last batch's rows
  int busy = 0;                // instances executing a batch (under mu)
  int instances = 1;
  uint64_t last_start_ns = 0;  // staggered dispatch (under mu): the last batch's start
  int last_rows = 0;           // rows of the last dispatched batch (under mu)
  double ema_exec_ns = 0;      // ... and an EMA of a batch's execution wall time
  std::vector<TensorDef> inputs, outputs;
  tcserve_exec_fn fn = nullptr;
  void* user = nullptr;
  // batcher
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::unique_ptr<PendingReq>> q;
  int q_rows = 0;
  bool stopping = false;
  std::vector<std::thread> workers;
  // stats
  std::mutex smu;
  uint64_t inference_count = 0, execution_count = 0, last_inference_ms = 0;
  Stat success, fail, queue, cin, cinf, cout;
  std::map<int, BatchStat> batch;
};

static size_t DtypeSize(const std::string& dt)
{
  if (dt == "BOOL" || dt == "INT8" || dt == "UINT8") return 1;
  if (dt == "INT16" || dt == "UINT16" || dt == "FP16" || dt == "BF16") return 2;
  if (dt == "INT32" || dt == "UINT32" || dt == "FP32") return 4;
  if (dt == "INT64" || dt == "UINT64" || dt == "FP64") return 8;
  return 0;
}

struct ShmEntry {
  uint64_t ptr = 0, bytes = 0;
  int device = 0;
  // one reference per queued/executing request that points into the region;
  // unregister waits for the requests to drop theirs before the caller unmaps
  std::shared_ptr<int> pin = std::make_shared<int>(0);
};

// [off, off + len) inside a region of `size` bytes, with no signed overflow:
// a negative byte size or offset is rejected before any arithmetic.
static bool ShmRangeOk(int64_t off, int64_t len, uint64_t size)
{
  if (off < 0 || len < 0) return false;
  return static_cast<uint64_t>(off) <= size && static_cast<uint64_t>(len) <= size - static_cast<uint64_t>(off);
}

// ---------------------------------------------------------------------------
class Loop {
 public:
  Loop(Server* srv, int idx) : srv_(srv), idx_(idx) {}
  bool Start(std::string* err);
  void Stop();
  void Post(std::function<void()> fn);
  void AddConn(int fd, bool http1 = false);
  void AddListener(int fd, uint64_t tag);
  Conn* Find(uint64_t id)
  {
    auto it = conns_.find(id);
    return it == conns_.end() ? nullptr : it->second.get();
  }
  void Flush(Conn* c);
  void Close(Conn* c);
  int idx() const { return idx_; }
  Server* srv() { return srv_; }
  int listen_fd = -1;       // only loop 0 accepts (gRPC)
  int http_listen_fd = -1;  // loop 0, KServe REST (tcserve_listen_http)

 private:
  void Run();
  void OnReadable(Conn* c);
  void DoAccept(bool http);
  Server* srv_;
  int idx_;
  int ep_ = -1, ev_ = -1;
  std::thread th_;
  std::atomic<bool> stop_{false};
  std::mutex mu_;
  std::deque<std::function<void()>> tasks_;
  std::unordered_map<uint64_t, std::unique_ptr<Conn>> conns_;
};

// Response compression for the native REST path (Accept-Encoding gzip /
// deflate).  Deflating a batch's responses inline would hold the batcher
// thread (the next batch waits behind zlib) and a loop thread would stall
// every connection on it, so the work goes to this small pool: two threads,
// started on first use, drained and joined when the server stops.
class CodecPool {
 public:
  ~CodecPool() { Stop(); }
  void Submit(std::function<void()> f)
  {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (!stop_) {
        if (th_.empty())
          for (int i = 0; i < 2; ++i)
            th_.emplace_back([this, i] {
              pthread_setname_np(pthread_self(), ("tcs-codec" + std::to_string(i)).c_str());
              Run();
            });
        q_.push_back(std::move(f));
        f = nullptr;
      }
    }
    if (f) {
      f();  // stopping: the pool no longer takes work, so the caller runs it (the connection still gets its reply)
      return;
    }
    cv_.notify_one();
  }
  // runs what is queued, then joins; later Submit()s run on their caller
  void Stop()
  {
    std::vector<std::thread> th;
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      th.swap(th_);  // under mu_: a concurrent Submit() sees either the running pool or stop_
    }
    cv_.notify_all();
    for (auto& t : th)
      if (t.joinable()) t.join();
  }

 private:
  void Run()
  {
    while (true) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;  // stopping and drained
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  std::vector<std::thread> th_;
  bool stop_ = false;
};

class Server {
 public:
  ~Server();
  bool Start(const std::string& host, int port, const std::string& up_host, int up_port, int io_threads,
             std::string* err);
  int port() const { return port_; }

  // transport hooks (loop thread)
  void OnHttpData(Conn* c);
  void RejectTooLarge(Conn* c);
  void OnRequestComplete(Conn* c, Stream* st);
  void OnStreamMessage(Conn* c, Stream* st, std::string&& msg);
  void OnStreamEnd(Conn* c, Stream* st);
  void OnStreamClosed(Conn* c, Stream* st);

  // response helpers (loop thread)
  void Reply(Conn* c, Stream* st, std::string* msg, int status, const std::string& message);
  void PostReply(Loop* loop, uint64_t conn_id, int32_t stream_id, std::string&& msg, int status,
                 const std::string& message);
  void PostHttp(Loop* loop, uint64_t conn_id, uint64_t seq, std::string&& bytes, bool close);
  bool ListenHttp(const std::string& host, int port, const std::string& up_host, int up_port, std::string* err);
  int http_port() const { return http_port_; }

  // native models / shm mirror
  int AddModel(std::unique_ptr<NativeModel> m, std::string* err);
  int RemoveModel(const std::string& name);
  void ShmAdd(int kind, const std::string& name, const ShmEntry& e);
  int ShmRemove(int kind, const std::string& name);
  int ShmBusy(int kind, uint64_t ptr);
  NativeModel* FindModel(const std::string& name);
  std::mutex models_mu;
  std::map<std::string, std::shared_ptr<NativeModel>> models;
  std::atomic<uint64_t> n_native{0}, n_proxied{0}, n_conns{0};
  // native REST requests whose body arrived compressed / whose response was compressed
  std::atomic<uint64_t> n_inflated{0}, n_deflated{0};

  std::vector<std::unique_ptr<Loop>> loops;
  std::atomic<uint64_t> next_conn_id{1};
  std::atomic<int> next_loop{0};

 private:
  bool TryNative(Conn* c, Stream* st, const char* msg, size_t len, std::string* owner);
  // (any thread: the connection is named by its loop and id)
  bool TryNativeHttp(Loop* loop, uint64_t conn_id, uint64_t seq, bool close, const std::string& name,
                     const std::string& version, std::string* body, size_t json_len, int resp_enc);
  void ProxyHttp(Loop* loop, uint64_t conn_id, uint64_t seq, bool close, std::string&& raw);
  void FailPending(PendingReq* pr, int grpc_status, int http_status, const std::string& msg);
  void Proxy(Conn* c, Stream* st, bool streaming);
  std::shared_ptr<tc::H2Channel> Upstream();
  void Worker(std::shared_ptr<NativeModel> m, int instance);
  void Execute(const std::shared_ptr<NativeModel>& ms, int instance, std::vector<std::unique_ptr<PendingReq>>& batch);
  static std::string HttpInferResponse(NativeModel* m, PendingReq* pr);

  int port_ = 0, http_port_ = 0;
  std::string up_host_, up_http_host_;
  int up_port_ = 0, up_http_port_ = 0;
  std::atomic<int> proxies_{0};  // in-flight HTTP proxy threads
  CodecPool codec_;              // REST response compression (off the batcher threads)
  std::mutex up_mu_;
  std::vector<std::shared_ptr<tc::H2Channel>> up_;
  std::atomic<uint32_t> up_rr_{0};
  std::mutex shm_mu_;
  std::map<std::string, ShmEntry> shm_[2];
  // unregistered regions that queued or executing requests still point into
  struct Draining {
    int kind;
    uint64_t ptr;
    std::shared_ptr<int> pin;
  };
  std::vector<Draining> draining_;
};

// ---------------------------------------------------------------------------
// nghttp2 server callbacks
// ---------------------------------------------------------------------------
static ssize_t ReadCb(nghttp2_session* session, int32_t stream_id, uint8_t* buf, size_t length, uint32_t* flags,
                      nghttp2_data_source* source, void* user)
{
  Conn* c = static_cast<Conn*>(user);
  auto it = c->streams.find(stream_id);
  if (it == c->streams.end()) {
    *flags |= NGHTTP2_DATA_FLAG_EOF;
    return 0;
  }
  Stream* st = it->second.get();
  size_t n = 0;
  while (n < length && !st->out.empty()) {
    std::string& f = st->out.front();
    size_t take = std::min(length - n, f.size() - st->out_pos);
    memcpy(buf + n, f.data() + st->out_pos, take);
    n += take;
    st->out_pos += take;
    if (st->out_pos == f.size()) {
      st->out.pop_front();
      st->out_pos = 0;
    }
  }
  if (st->out.empty() && st->finish) {
    *flags |= NGHTTP2_DATA_FLAG_EOF;
    if (!st->trailers_sent) {
      *flags |= NGHTTP2_DATA_FLAG_NO_END_STREAM;
      std::string code = std::to_string(st->status);
      std::vector<nghttp2_nv> nv;
      auto mk = [](const std::string& k, const std::string& v) {
        nghttp2_nv x;
        x.name = (uint8_t*)k.data();
        x.value = (uint8_t*)v.data();
        x.namelen = k.size();
        x.valuelen = v.size();
        x.flags = NGHTTP2_NV_FLAG_NONE;
        return x;
      };
      static const std::string kStatus = "grpc-status", kMsg = "grpc-message";
      std::string msg = tc::UrlEncode(st->message);
      nv.push_back(mk(kStatus, code));
      if (!st->message.empty()) nv.push_back(mk(kMsg, msg));
      nghttp2_submit_trailer(session, stream_id, nv.data(), nv.size());  // copies nv
      st->trailers_sent = true;
    }
    return static_cast<ssize_t>(n);
  }
  if (n == 0) {
    st->deferred = true;
    return NGHTTP2_ERR_DEFERRED;
  }
  return static_cast<ssize_t>(n);
}

static int OnBeginHeaders(nghttp2_session*, const nghttp2_frame* frame, void* user)
{
  Conn* c = static_cast<Conn*>(user);
  if (frame->hd.type == NGHTTP2_HEADERS && frame->headers.cat == NGHTTP2_HCAT_REQUEST) {
    std::unique_ptr<Stream> st(new Stream());
    st->id = frame->hd.stream_id;
    c->streams[st->id] = std::move(st);
  }
  return 0;
}

static int OnHeader(nghttp2_session*, const nghttp2_frame* frame, const uint8_t* name, size_t namelen,
                    const uint8_t* value, size_t valuelen, uint8_t, void* user)
{
  Conn* c = static_cast<Conn*>(user);
  auto it = c->streams.find(frame->hd.stream_id);
  if (it == c->streams.end()) return 0;
  std::string k(reinterpret_cast<const char*>(name), namelen), v(reinterpret_cast<const char*>(value), valuelen);
  if (k == ":path") {
    it->second->path = v;
    it->second->streaming_rpc = v == "/inference.GRPCInferenceService/ModelStreamInfer";
  } else if (!k.empty() && k[0] != ':' && k != "content-type" && k != "te" && k != "grpc-accept-encoding" &&
             k != "user-agent" && k != "grpc-timeout" && k != "content-length") {
    it->second->meta.emplace_back(k, v);
  }
  return 0;
}

// Pop complete gRPC messages off the stream's input buffer.
static bool PopMessages(Stream* st, std::vector<std::string>* msgs, std::string* err)
{
  size_t pos = 0;
  bool gz = false;
  for (const auto& kv : st->meta)
    if (kv.first == "grpc-encoding" && kv.second != "identity") gz = true;
  while (st->inbuf.size() - pos >= 5) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(st->inbuf.data() + pos);
    const uint32_t n = (uint32_t(p[1]) << 24) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 8) | p[4];
    if (st->inbuf.size() - pos - 5 < n) break;
    if (p[0] && gz) {
      std::string dec;
      if (!tc::Decompress(st->inbuf.substr(pos + 5, n), &dec)) {
        *err = "failed to decompress request message";
        return false;
      }
      msgs->push_back(std::move(dec));
    } else {
      msgs->emplace_back(st->inbuf.data() + pos + 5, n);
    }
    pos += 5 + n;
  }
  st->inbuf.erase(0, pos);
  return true;
}

static int OnDataChunk(nghttp2_session*, uint8_t, int32_t stream_id, const uint8_t* data, size_t len, void* user)
{
  Conn* c = static_cast<Conn*>(user);
  auto it = c->streams.find(stream_id);
  if (it == c->streams.end()) return 0;
  Stream* st = it->second.get();
  const bool was_short = st->inbuf.size() < 5;
  st->inbuf.append(reinterpret_cast<const char*>(data), len);
  if (was_short && !st->streaming_rpc && st->inbuf.size() >= 5) {
    // unary: size the buffer for the whole message now (no regrowth copies)
    const uint8_t* p = reinterpret_cast<const uint8_t*>(st->inbuf.data());
    const size_t n = (size_t(p[1]) << 24) | (size_t(p[2]) << 16) | (size_t(p[3]) << 8) | p[4];
    if (n < (size_t(1) << 31)) st->inbuf.reserve(5 + n);
  }
  if (st->streaming_rpc) {
    std::vector<std::string> msgs;
    std::string err;
    if (!PopMessages(st, &msgs, &err)) return 0;
    for (auto& m : msgs) c->loop->srv()->OnStreamMessage(c, st, std::move(m));
  }
  return 0;
}

static int OnFrameRecv(nghttp2_session*, const nghttp2_frame* frame, void* user)
{
  Conn* c = static_cast<Conn*>(user);
  if (frame->hd.type != NGHTTP2_HEADERS && frame->hd.type != NGHTTP2_DATA) return 0;
  auto it = c->streams.find(frame->hd.stream_id);
  if (it == c->streams.end()) return 0;
  Stream* st = it->second.get();
  if (frame->hd.type == NGHTTP2_HEADERS && st->streaming_rpc && !st->started) {
    c->loop->srv()->OnStreamMessage(c, st, std::string());  // opens the upstream call (empty = open only)
  }
  if (frame->hd.flags & NGHTTP2_FLAG_END_STREAM) {
    st->end_stream = true;
    if (st->streaming_rpc) c->loop->srv()->OnStreamEnd(c, st);
    else c->loop->srv()->OnRequestComplete(c, st);
  }
  return 0;
}

static int OnStreamClose(nghttp2_session*, int32_t stream_id, uint32_t, void* user)
{
  Conn* c = static_cast<Conn*>(user);
  auto it = c->streams.find(stream_id);
  if (it == c->streams.end()) return 0;
  c->loop->srv()->OnStreamClosed(c, it->second.get());
  c->streams.erase(it);
  return 0;
}

// ---------------------------------------------------------------------------
// Loop
// ---------------------------------------------------------------------------
bool Loop::Start(std::string* err)
{
  ep_ = epoll_create1(EPOLL_CLOEXEC);
  ev_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (ep_ < 0 || ev_ < 0) {
    *err = "epoll/eventfd failed";
    return false;
  }
  epoll_event e{};
  e.events = EPOLLIN;
  e.data.u64 = 0;  // 0 = eventfd
  epoll_ctl(ep_, EPOLL_CTL_ADD, ev_, &e);
  if (listen_fd >= 0) {
    e.events = EPOLLIN;
    e.data.u64 = 1;  // 1 = listen socket
    epoll_ctl(ep_, EPOLL_CTL_ADD, listen_fd, &e);
  }
  th_ = std::thread(&Loop::Run, this);
  return true;
}

void Loop::Stop()
{
  stop_ = true;
  uint64_t one = 1;
  if (ev_ >= 0) (void)!write(ev_, &one, 8);
  if (th_.joinable()) th_.join();
  for (auto& kv : conns_) {
    if (kv.second->s) nghttp2_session_del(kv.second->s);
    close(kv.second->fd);
  }
  conns_.clear();
  if (ep_ >= 0) close(ep_);
  if (ev_ >= 0) close(ev_);
}

void Loop::Post(std::function<void()> fn)
{
  {
    std::lock_guard<std::mutex> lk(mu_);
    tasks_.push_back(std::move(fn));
  }
  uint64_t one = 1;
  (void)!write(ev_, &one, 8);
}

void Loop::AddListener(int fd, uint64_t tag)
{
  epoll_event e{};
  e.events = EPOLLIN;
  e.data.u64 = tag;
  epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &e);
}

void Loop::AddConn(int fd, bool http1)
{
  std::unique_ptr<Conn> c(new Conn());
  c->id = srv_->next_conn_id++;
  c->fd = fd;
  c->loop = this;
  c->http1 = http1;
  if (http1) {
    epoll_event e{};
    e.events = EPOLLIN;
    e.data.u64 = c->id + 16;
    epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &e);
    conns_[c->id] = std::move(c);
    srv_->n_conns++;
    return;
  }
  nghttp2_session_callbacks* cbs;
  nghttp2_session_callbacks_new(&cbs);
  nghttp2_session_callbacks_set_on_begin_headers_callback(cbs, OnBeginHeaders);
  nghttp2_session_callbacks_set_on_header_callback(cbs, OnHeader);
  nghttp2_session_callbacks_set_on_data_chunk_recv_callback(cbs, OnDataChunk);
  nghttp2_session_callbacks_set_on_frame_recv_callback(cbs, OnFrameRecv);
  nghttp2_session_callbacks_set_on_stream_close_callback(cbs, OnStreamClose);
  nghttp2_session_server_new(&c->s, cbs, c.get());
  nghttp2_session_callbacks_del(cbs);
  nghttp2_settings_entry iv[3] = {{NGHTTP2_SETTINGS_MAX_CONCURRENT_STREAMS, 4096},
                                  {NGHTTP2_SETTINGS_INITIAL_WINDOW_SIZE, (1u << 31) - 1},
                                  {NGHTTP2_SETTINGS_MAX_FRAME_SIZE, 1u << 20}};
  nghttp2_submit_settings(c->s, NGHTTP2_FLAG_NONE, iv, 3);
  nghttp2_session_set_local_window_size(c->s, NGHTTP2_FLAG_NONE, 0, (1 << 30));
  epoll_event e{};
  e.events = EPOLLIN;
  e.data.u64 = c->id + 16;  // ids below 16 are reserved
  epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &e);
  Conn* raw = c.get();
  conns_[c->id] = std::move(c);
  srv_->n_conns++;
  Flush(raw);
}

void Loop::Close(Conn* c)
{
  epoll_ctl(ep_, EPOLL_CTL_DEL, c->fd, nullptr);
  for (auto& kv : c->streams) srv_->OnStreamClosed(c, kv.second.get());
  c->streams.clear();
  if (c->s) nghttp2_session_del(c->s);
  close(c->fd);
  conns_.erase(c->id);
}

void Loop::Flush(Conn* c)
{
  while (true) {
    if (c->sendpos == c->sendbuf.size() && c->http1) {
      c->sendbuf.clear();
      c->sendpos = 0;
      break;
    }
    if (c->sendpos == c->sendbuf.size()) {
      c->sendbuf.clear();
      c->sendpos = 0;
      const uint8_t* data;
      ssize_t n;
      while ((n = nghttp2_session_mem_send(c->s, &data)) > 0) {
        c->sendbuf.append(reinterpret_cast<const char*>(data), n);
        if (c->sendbuf.size() > (1 << 20)) break;
      }
      if (n < 0) {
        c->closing = true;
        break;
      }
      if (c->sendbuf.empty()) break;
    }
    ssize_t w = send(c->fd, c->sendbuf.data() + c->sendpos, c->sendbuf.size() - c->sendpos, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      if (errno == EINTR) continue;
      c->closing = true;
      break;
    }
    c->sendpos += w;
  }
  const bool pending = c->sendpos < c->sendbuf.size();
  if (pending != c->want_write && !c->closing) {
    epoll_event e{};
    e.events = EPOLLIN | (pending ? static_cast<uint32_t>(EPOLLOUT) : 0u);
    e.data.u64 = c->id + 16;
    epoll_ctl(ep_, EPOLL_CTL_MOD, c->fd, &e);
    c->want_write = pending;
  }
  if (c->http1) {
    // Connection: close -> close once every response before it has gone out
    if (c->closing || (c->close_after && !pending && c->resp_seq == c->req_seq)) Close(c);
    return;
  }
  if (c->closing ||
      (!nghttp2_session_want_read(c->s) && !nghttp2_session_want_write(c->s) && !pending)) {
    Close(c);
  }
}

void Loop::OnReadable(Conn* c)
{
  uint8_t buf[65536];
  while (true) {
    ssize_t n = recv(c->fd, buf, sizeof(buf), 0);
    if (n > 0 && c->http1) {
      c->hin.append(reinterpret_cast<const char*>(buf), n);
      continue;
    }
    if (n > 0) {
      ssize_t r = nghttp2_session_mem_recv(c->s, buf, n);
      if (r < 0) {
        c->closing = true;
        break;
      }
      continue;
    }
    if (n == 0) {
      c->closing = true;
      break;
    }
    if (errno == EAGAIN || errno == EWOULDBLOCK) break;
    if (errno == EINTR) continue;
    c->closing = true;
    break;
  }
  if (c->http1 && !c->hin.empty() && !c->closing) {
    const uint64_t id = c->id;
    srv_->OnHttpData(c);
    c = Find(id);
    if (!c) return;
  }
  if (c->closing) {
    Close(c);
    return;
  }
  Flush(c);
}

void Loop::DoAccept(bool http)
{
  while (true) {
    int fd = accept4(http ? http_listen_fd : listen_fd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
    if (fd < 0) break;
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    const int li = srv_->next_loop++ % static_cast<int>(srv_->loops.size());
    Loop* l = srv_->loops[li].get();
    if (l == this) AddConn(fd, http);
    else l->Post([l, fd, http] { l->AddConn(fd, http); });
  }
}

void Loop::Run()
{
  pthread_setname_np(pthread_self(), ("tcs-loop" + std::to_string(idx_)).c_str());
  epoll_event evs[64];
  while (!stop_) {
    int n = epoll_wait(ep_, evs, 64, 200);
    for (int i = 0; i < n; ++i) {
      const uint64_t tag = evs[i].data.u64;
      if (tag == 0) {
        uint64_t v;
        (void)!read(ev_, &v, 8);
        std::deque<std::function<void()>> tasks;
        {
          std::lock_guard<std::mutex> lk(mu_);
          tasks.swap(tasks_);
        }
        for (auto& t : tasks) t();
      } else if (tag == 1 || tag == 2) {
        DoAccept(tag == 2);
      } else {
        Conn* c = Find(tag - 16);
        if (!c) continue;
        if (evs[i].events & (EPOLLERR | EPOLLHUP)) {
          Close(c);
          continue;
        }
        if (evs[i].events & EPOLLIN) {
          OnReadable(c);
          c = Find(tag - 16);
        }
        if (c && (evs[i].events & EPOLLOUT)) Flush(c);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Server
// ---------------------------------------------------------------------------
bool Server::Start(const std::string& host, int port, const std::string& up_host, int up_port, int io_threads,
                   std::string* err)
{
  up_host_ = up_host;
  up_port_ = up_port;
  int fd = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(port));
  if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) a.sin_addr.s_addr = htonl(INADDR_ANY);
  if (bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || listen(fd, 1024) != 0) {
    *err = "cannot bind/listen on port " + std::to_string(port) + ": " + strerror(errno);
    close(fd);
    return false;
  }
  socklen_t al = sizeof(a);
  getsockname(fd, reinterpret_cast<sockaddr*>(&a), &al);
  port_ = ntohs(a.sin_port);
  const int n = std::max(1, io_threads);
  for (int i = 0; i < n; ++i) loops.emplace_back(new Loop(this, i));
  loops[0]->listen_fd = fd;
  for (auto& l : loops)
    if (!l->Start(err)) return false;
  return true;
}

Server::~Server()
{
  std::vector<std::shared_ptr<NativeModel>> ms;
  {
    std::lock_guard<std::mutex> lk(models_mu);
    for (auto& kv : models) ms.push_back(kv.second);
    models.clear();
  }
  for (auto& m : ms) {
    {
      std::lock_guard<std::mutex> lk(m->mu);
      m->stopping = true;
    }
    m->cv.notify_all();
    for (auto& t : m->workers)
      if (t.joinable()) t.join();
  }
  codec_.Stop();  // queued compressed responses still post to the loops
  for (int i = 0; i < 3000 && proxies_.load() > 0; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(1));
  for (auto& l : loops) l->Stop();
  if (!loops.empty() && loops[0]->listen_fd >= 0) close(loops[0]->listen_fd);
  if (!loops.empty() && loops[0]->http_listen_fd >= 0) close(loops[0]->http_listen_fd);
  loops.clear();
  std::lock_guard<std::mutex> lk(up_mu_);
  up_.clear();
}

std::shared_ptr<tc::H2Channel> Server::Upstream()
{
  std::lock_guard<std::mutex> lk(up_mu_);
  if (up_.empty()) up_.resize(4);
  const size_t i = up_rr_++ % up_.size();
  if (!up_[i] || !up_[i]->Healthy()) {
    std::string err;
    tc::H2ChannelOptions o;
    up_[i] = tc::H2Channel::Create(up_host_, up_port_, o, &err);
  }
  return up_[i];
}

void Server::Reply(Conn* c, Stream* st, std::string* msg, int status, const std::string& message)
{
  if (msg) {
    std::string framed;
    tc::GrpcFrame(*msg, tc::GrpcCompression::NONE, &framed);
    st->out.push_back(std::move(framed));
  }
  if (status >= 0) {
    st->finish = true;
    st->status = status;
    st->message = message;
  }
  if (!st->response_submitted) {
    nghttp2_nv hdrs[2];
    static const char s200[] = "200", ctype[] = "application/grpc";
    hdrs[0] = {(uint8_t*)":status", (uint8_t*)s200, 7, 3, NGHTTP2_NV_FLAG_NONE};
    hdrs[1] = {(uint8_t*)"content-type", (uint8_t*)ctype, 12, sizeof(ctype) - 1, NGHTTP2_NV_FLAG_NONE};
    nghttp2_data_provider prd;
    prd.source.ptr = nullptr;
    prd.read_callback = ReadCb;
    nghttp2_submit_response(c->s, st->id, hdrs, 2, &prd);
    st->response_submitted = true;
  } else if (st->deferred) {
    st->deferred = false;
    nghttp2_session_resume_data(c->s, st->id);
  }
}

void Server::PostReply(Loop* loop, uint64_t conn_id, int32_t stream_id, std::string&& msg, int status,
                       const std::string& message)
{
  auto m = std::make_shared<std::string>(std::move(msg));
  loop->Post([this, loop, conn_id, stream_id, m, status, message] {
    Conn* c = loop->Find(conn_id);
    if (!c) return;
    auto it = c->streams.find(stream_id);
    if (it == c->streams.end()) return;
    Reply(c, it->second.get(), status == kOk ? m.get() : nullptr, status, message);
    loop->Flush(c);
  });
}

// ---------------------------------------------------------------------------
// KServe REST (HTTP/1.1) front end: POST /v2/models/<m>[/versions/<v>]/infer
// for native models with binary-tensor or shared-memory I/O runs on the same
// batcher as gRPC; every other request is relayed byte-for-byte to the
// aiohttp server behind it (one upstream connection per relayed request).
// ---------------------------------------------------------------------------
namespace {

std::string Lower(std::string v)
{
  for (auto& ch : v) ch = static_cast<char>(tolower(static_cast<unsigned char>(ch)));
  return v;
}

std::string HttpStatusLine(int code)
{
  switch (code) {
    case 200: return "HTTP/1.1 200 OK\r\n";
    case 400: return "HTTP/1.1 400 Bad Request\r\n";
    case 500: return "HTTP/1.1 500 Internal Server Error\r\n";
    case 502: return "HTTP/1.1 502 Bad Gateway\r\n";
    case 413: return "HTTP/1.1 413 Payload Too Large\r\n";
    case 503: return "HTTP/1.1 503 Service Unavailable\r\n";
    default: return "HTTP/1.1 " + std::to_string(code) + " Error\r\n";
  }
}

std::string HttpError(int code, const std::string& msg, bool close)
{
  std::string body = "{\"error\":";
  tc::json::AppendEscapedString(&body, msg);
  body += "}";
  std::string r = HttpStatusLine(code);
  r += "Content-Type: application/json\r\nContent-Length: " + std::to_string(body.size()) + "\r\n";
  if (close) r += "Connection: close\r\n";
  r += "\r\n";
  return r + body;
}

struct HttpHead {
  std::string method, target;
  std::vector<std::pair<std::string, std::string>> headers;  // lower-case names
  size_t head_len = 0;
  const std::string* Get(const char* name) const
  {
    for (const auto& kv : headers)
      if (kv.first == name) return &kv.second;
    return nullptr;
  }
};

// Parse a request head ending at "\r\n\r\n"; 0 = need more, -1 = malformed, 1 = ok.
int ParseHead(const std::string& in, HttpHead* h)
{
  const size_t end = in.find("\r\n\r\n");
  if (end == std::string::npos) return in.size() > (1u << 20) ? -1 : 0;
  h->head_len = end + 4;
  size_t pos = in.find("\r\n");
  const std::string line = in.substr(0, pos);
  const size_t sp1 = line.find(' '), sp2 = line.rfind(' ');
  if (sp1 == std::string::npos || sp2 == sp1) return -1;
  h->method = line.substr(0, sp1);
  h->target = line.substr(sp1 + 1, sp2 - sp1 - 1);
  pos += 2;
  while (pos < end) {
    const size_t eol = in.find("\r\n", pos);
    const std::string l = in.substr(pos, eol - pos);
    const size_t colon = l.find(':');
    if (colon != std::string::npos) {
      size_t v = colon + 1;
      while (v < l.size() && (l[v] == ' ' || l[v] == '\t')) ++v;
      size_t ve = l.size();
      while (ve > v && (l[ve - 1] == ' ' || l[ve - 1] == '\t')) --ve;
      h->headers.emplace_back(Lower(l.substr(0, colon)), l.substr(v, ve - v));
    }
    pos = eol + 2;
  }
  return 1;
}

// Decode a chunked body starting at `from`; 0 = need more, -1 = malformed, else bytes consumed.
// Largest request body tcserve buffers (Content-Length or de-chunked); larger
// requests get 413 and the connection is closed.  KServe gRPC messages are
// capped at INT32_MAX too (reference src/c++/library/common.h:53).
constexpr uint64_t kMaxHttpBody = 0x7fffffffull;
// compressed REST bodies at least this large are inflated on the codec pool, not the loop thread
constexpr size_t kInflateOnLoopMax = 64 * 1024;

// returns bytes consumed, 0 = need more input, -1 = malformed, -2 = too large
long DecodeChunked(const std::string& in, size_t from, std::string* body)
{
  size_t pos = from;
  body->clear();
  while (true) {
    const size_t eol = in.find("\r\n", pos);
    if (eol == std::string::npos) return 0;
    char* e = nullptr;
    const unsigned long n = strtoul(in.c_str() + pos, &e, 16);
    if (e == in.c_str() + pos) return -1;
    pos = eol + 2;
    if (n == 0) {
      const size_t fin = in.find("\r\n", pos);  // (no trailers expected)
      if (fin == std::string::npos) return 0;
      return static_cast<long>(fin + 2 - from);
    }
    if (n > kMaxHttpBody || body->size() + n > kMaxHttpBody) return -2;
    if (in.size() < pos || n + 2 > in.size() - pos) return 0;
    body->append(in, pos, n);
    pos += n + 2;
  }
}

// /v2/models/<m>[/versions/<v>]/infer -> (m, v)
bool InferTarget(const std::string& target, std::string* model, std::string* version)
{
  static const std::string pre = "/v2/models/", suf = "/infer";
  if (target.compare(0, pre.size(), pre) != 0 || target.size() <= pre.size() + suf.size() ||
      target.compare(target.size() - suf.size(), suf.size(), suf) != 0 || target.find('?') != std::string::npos)
    return false;
  const std::string mid = target.substr(pre.size(), target.size() - pre.size() - suf.size());
  const size_t vpos = mid.find("/versions/");
  if (vpos == std::string::npos) {
    if (mid.find('/') != std::string::npos) return false;
    *model = mid;
    version->clear();
  } else {
    *model = mid.substr(0, vpos);
    *version = mid.substr(vpos + 10);
    if (model->find('/') != std::string::npos || version->find('/') != std::string::npos) return false;
  }
  return !model->empty();
}

}  // namespace

void Server::RejectTooLarge(Conn* c)
{
  const uint64_t seq = c->req_seq++;
  c->close_after = true;
  c->hin.clear();
  PostHttp(c->loop, c->id, seq, HttpError(413, "request body exceeds " + std::to_string(kMaxHttpBody) + " bytes", true),
           true);
}

// Content-Encoding of a request body: 0 identity, 1 gzip, 2 deflate, -1 other (proxied).
static int ContentCoding(const std::string* ce)
{
  if (!ce) return 0;
  const std::string v = Lower(*ce);
  if (v.empty() || v == "identity") return 0;
  if (v == "gzip" || v == "x-gzip") return 1;
  if (v == "deflate") return 2;
  return -1;
}

// Response coding from Accept-Encoding: gzip preferred, then deflate (q=0 excluded).
static int AcceptCoding(const std::string* ae)
{
  if (!ae) return 0;
  const std::string v = Lower(*ae);
  auto offered = [&](const char* tok) {
    size_t p = 0;
    const size_t n = strlen(tok);
    while ((p = v.find(tok, p)) != std::string::npos) {
      const bool start = p == 0 || v[p - 1] == ',' || v[p - 1] == ' ';
      size_t e = p + n;
      while (e < v.size() && v[e] == ' ') ++e;
      const bool end = e == v.size() || v[e] == ',' || v[e] == ';';
      if (start && end) {
        const size_t q = v.find("q=", e);
        const size_t comma = v.find(',', e);
        if (q != std::string::npos && (comma == std::string::npos || q < comma)) return strtod(v.c_str() + q + 2, nullptr) > 0;
        return true;
      }
      p = e;
    }
    return false;
  };
  if (offered("gzip")) return 1;
  if (offered("deflate")) return 2;
  return 0;
}

// zlib/gzip inflate (header auto-detected) with an output cap (no decompression bombs).
static bool InflateBounded(const std::string& in, uint64_t cap, std::string* out)
{
  z_stream zs;
  memset(&zs, 0, sizeof(zs));
  if (inflateInit2(&zs, 15 | 32) != Z_OK) return false;
  out->clear();
  size_t pos = 0;
  char buf[1 << 16];
  int rc = Z_OK;
  while (rc != Z_STREAM_END) {
    if (zs.avail_in == 0) {
      if (pos >= in.size()) break;
      const size_t take = std::min<size_t>(in.size() - pos, 1u << 30);
      zs.next_in = reinterpret_cast<Bytef*>(const_cast<char*>(in.data() + pos));
      zs.avail_in = static_cast<uInt>(take);
      pos += take;
    }
    zs.next_out = reinterpret_cast<Bytef*>(buf);
    zs.avail_out = sizeof(buf);
    rc = inflate(&zs, Z_NO_FLUSH);
    if (rc != Z_OK && rc != Z_STREAM_END) break;
    out->append(buf, sizeof(buf) - zs.avail_out);
    if (out->size() > cap) {
      rc = Z_DATA_ERROR;
      break;
    }
  }
  inflateEnd(&zs);
  return rc == Z_STREAM_END;
}

// gzip (enc 1) or zlib "deflate" (enc 2) of parts, fastest level.
static bool DeflateParts(const std::vector<std::pair<const char*, size_t>>& parts, int enc, std::string* out)
{
  z_stream zs;
  memset(&zs, 0, sizeof(zs));
  if (deflateInit2(&zs, Z_BEST_SPEED, Z_DEFLATED, enc == 1 ? 15 | 16 : 15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
  size_t total = 0;
  for (const auto& p : parts) total += p.second;
  out->clear();
  out->reserve(deflateBound(&zs, static_cast<uLong>(total)) + 64);
  char buf[1 << 16];
  bool ok = true;
  for (size_t i = 0; i < parts.size() && ok; ++i) {
    const char* d = parts[i].first;
    size_t left = parts[i].second;
    const bool last_part = i + 1 == parts.size();
    do {
      const size_t take = std::min<size_t>(left, 1u << 30);
      zs.next_in = reinterpret_cast<Bytef*>(const_cast<char*>(d));
      zs.avail_in = static_cast<uInt>(take);
      d += take;
      left -= take;
      const int flush = (last_part && left == 0) ? Z_FINISH : Z_NO_FLUSH;
      int rc;
      do {
        zs.next_out = reinterpret_cast<Bytef*>(buf);
        zs.avail_out = sizeof(buf);
        rc = deflate(&zs, flush);
        if (rc == Z_STREAM_ERROR) {
          ok = false;
          break;
        }
        out->append(buf, sizeof(buf) - zs.avail_out);
      } while (zs.avail_out == 0);
    } while (left > 0 && ok);
  }
  if (parts.empty() && ok) {
    zs.avail_in = 0;
    int rc;
    do {
      zs.next_out = reinterpret_cast<Bytef*>(buf);
      zs.avail_out = sizeof(buf);
      rc = deflate(&zs, Z_FINISH);
      out->append(buf, sizeof(buf) - zs.avail_out);
    } while (rc == Z_OK);
  }
  deflateEnd(&zs);
  return ok;
}

void Server::OnHttpData(Conn* c)
{
  while (!c->hin.empty() && !c->close_after) {
    HttpHead h;
    const int ph = ParseHead(c->hin, &h);
    if (ph == 0) return;
    if (ph < 0) {
      c->closing = true;
      return;
    }
    std::string body;
    size_t consumed = h.head_len;
    const std::string* te = h.Get("transfer-encoding");
    const std::string* cl = h.Get("content-length");
    bool rebuilt = false;
    if (te && Lower(*te).find("chunked") != std::string::npos) {
      const long n = DecodeChunked(c->hin, h.head_len, &body);
      if (n == 0) return;
      if (n == -2) return RejectTooLarge(c);
      if (n < 0) {
        c->closing = true;
        return;
      }
      consumed += static_cast<size_t>(n);
      rebuilt = true;  // relay with Content-Length instead of chunks
    } else if (cl) {
      const uint64_t n = strtoull(cl->c_str(), nullptr, 10);
      if (n > kMaxHttpBody) return RejectTooLarge(c);
      if (c->hin.size() < h.head_len + n) return;
      body.assign(c->hin, h.head_len, n);
      consumed += n;
    }
    const std::string* conn_hdr = h.Get("connection");
    const bool close = conn_hdr && Lower(*conn_hdr) == "close";
    const uint64_t seq = c->req_seq++;
    if (close) c->close_after = true;
    std::string model, version;
    const std::string* ihcl = h.Get("inference-header-content-length");
    const std::string* ce = h.Get("content-encoding");
    const std::string* ae = h.Get("accept-encoding");
    bool handled = false;
    if (h.method == "POST" && InferTarget(h.target, &model, &version) && ihcl) {
      // KServe REST compression (reference http_client.cc:143-232, Python
      // _client.py:1440-1460): a gzip / deflate request body is inflated here
      // and the response compressed to the client's Accept-Encoding, so a
      // compressed request stays on the native path.  Inference-Header-Content-Length
      // counts the uncompressed JSON header in both directions.
      const int req_enc = ContentCoding(ce);
      const int resp_enc = AcceptCoding(ae);
      const size_t jl = strtoull(ihcl->c_str(), nullptr, 10);
      if (req_enc > 0 && body.size() >= kInflateOnLoopMax) {
        // a large compressed body is inflated on the codec pool, not here (a
        // gzip client would stall every connection of this loop); the pool
        // thread then takes the native path, or relays the original request
        std::string head;
        if (rebuilt) {
          head = h.method + " " + h.target + " HTTP/1.1\r\n";
          for (const auto& kv : h.headers)
            if (kv.first != "transfer-encoding" && kv.first != "content-length")
              head += kv.first + ": " + kv.second + "\r\n";
          head += "Content-Length: " + std::to_string(body.size()) + "\r\n\r\n";
        } else {
          head.assign(c->hin, 0, h.head_len);
        }
        Loop* loop = c->loop;
        const uint64_t conn_id = c->id;
        auto zbody = std::make_shared<std::string>(std::move(body));
        codec_.Submit([this, loop, conn_id, seq, close, model, version, jl, resp_enc, head, zbody] {
          std::string plain;
          bool done = false;
          if (InflateBounded(*zbody, kMaxHttpBody, &plain)) {
            n_inflated++;
            if (jl <= plain.size()) done = TryNativeHttp(loop, conn_id, seq, close, model, version, &plain, jl, resp_enc);
          }
          if (!done) ProxyHttp(loop, conn_id, seq, close, head + *zbody);
        });
        handled = true;
      } else {
        std::string plain;
        bool ok = req_enc >= 0;
        if (ok && req_enc > 0) {
          ok = InflateBounded(body, kMaxHttpBody, &plain);
          if (ok) n_inflated++;
        }
        if (ok) {
          std::string& b = req_enc > 0 ? plain : body;
          if (jl <= b.size()) handled = TryNativeHttp(c->loop, c->id, seq, close, model, version, &b, jl, resp_enc);
        }
      }
    }
    if (!handled) {
      std::string raw;
      if (rebuilt) {
        // head without Transfer-Encoding + Content-Length, then the decoded body
        raw = h.method + " " + h.target + " HTTP/1.1\r\n";
        const std::string head = c->hin.substr(0, h.head_len);
        for (const auto& kv : h.headers)
          if (kv.first != "transfer-encoding" && kv.first != "content-length") raw += kv.first + ": " + kv.second + "\r\n";
        raw += "Content-Length: " + std::to_string(body.size()) + "\r\n\r\n" + body;
      } else {
        raw.assign(c->hin, 0, consumed);
      }
      ProxyHttp(c->loop, c->id, seq, close, std::move(raw));
    }
    c->hin.erase(0, consumed);
  }
}

bool Server::TryNativeHttp(Loop* loop, uint64_t conn_id, uint64_t seq, bool close, const std::string& name, const std::string& version,
                           std::string* body, size_t json_len, int resp_enc)
{
  std::shared_ptr<NativeModel> m;
  {
    std::lock_guard<std::mutex> lk(models_mu);
    auto it = models.find(name);
    if (it == models.end()) return false;
    m = it->second;
  }
  if (!version.empty() && version != m->version) return false;
  namespace js = tc::json;
  js::Value root;
  std::string perr;
  if (!js::Parse(body->data(), json_len, &root, &perr) || !root.IsObject()) return false;
  bool binary_out_default = false;
  if (const js::Value* params = root.Find("parameters")) {
    for (const auto& kv : params->Members()) {
      if (kv.first == "binary_data_output") binary_out_default = kv.second.AsBool();
      else if (kv.first != "priority" && kv.first != "timeout") return false;  // sequences etc.: Python server
    }
  }
  const js::Value* inputs = root.Find("inputs");
  if (!inputs || !inputs->IsArray() || inputs->Size() != m->inputs.size()) return false;
  std::unique_ptr<PendingReq> pr(new PendingReq());
  pr->http = true;
  pr->http_seq = seq;
  pr->http_close = close;
  pr->http_resp_enc = resp_enc;
  pr->conn_id = conn_id;
  pr->loop = loop;
  pr->stream_id = 0;
  if (const js::Value* id = root.Find("id")) pr->id = id->AsString();
  pr->t_arrive = NowNs();
  pr->in.resize(m->inputs.size());
  pr->rows = -1;
  size_t data_off = json_len;
  auto fail = [&](const std::string& msg) {
    PostHttp(loop, conn_id, seq, HttpError(400, msg, close), close);
    std::lock_guard<std::mutex> lk(m->smu);
    m->fail.count++;
    m->fail.ns += NowNs() - pr->t_arrive;
    return true;
  };
  auto lookup = [&](const std::string& region, ShmEntry* e) {
    std::lock_guard<std::mutex> lk(shm_mu_);
    for (int kk = 0; kk < 2; ++kk) {
      auto it = shm_[kk].find(region);
      if (it != shm_[kk].end()) {
        *e = it->second;
        return kk;
      }
    }
    return -1;
  };
  std::vector<bool> seen(m->inputs.size(), false);
  for (const js::Value& t : inputs->Elements()) {
    const js::Value* nm = t.Find("name");
    const js::Value* dt = t.Find("datatype");
    const js::Value* shape = t.Find("shape");
    if (!nm || !dt || !shape || !shape->IsArray() || t.Find("data")) return false;  // JSON tensor data: Python
    int idx = -1;
    for (size_t k = 0; k < m->inputs.size(); ++k)
      if (m->inputs[k].name == nm->AsString()) idx = static_cast<int>(k);
    if (idx < 0) return false;
    if (seen[idx]) return fail("input '" + nm->AsString() + "' is specified more than once");
    seen[idx] = true;
    const TensorDef& d = m->inputs[idx];
    if (dt->AsString() != d.dtype) return false;
    if (shape->Size() != d.dims.size() + (m->max_batch > 0 ? 1 : 0)) return false;
    int rows = 1;
    size_t off = 0;
    if (m->max_batch > 0) {
      rows = static_cast<int>((*shape)[0].AsInt());
      off = 1;
    }
    for (size_t k = 0; k < d.dims.size(); ++k)
      if ((*shape)[k + off].AsInt() != d.dims[k]) return false;
    if (rows < 1 || (m->max_batch > 0 && rows > m->max_batch)) return false;
    if (pr->rows >= 0 && pr->rows != rows) return false;
    pr->rows = rows;
    const uint64_t need = static_cast<uint64_t>(rows) * d.sample_bytes;
    std::string region;
    int64_t rbytes = 0, roff = 0, bsize = -1;
    bool has_shm = false;
    if (const js::Value* tp = t.Find("parameters")) {
      for (const auto& kv : tp->Members()) {
        if (kv.first == "shared_memory_region") {
          region = kv.second.AsString();
          has_shm = true;
        } else if (kv.first == "shared_memory_byte_size") {
          rbytes = kv.second.AsInt();
        } else if (kv.first == "shared_memory_offset") {
          roff = kv.second.AsInt();
        } else if (kv.first == "binary_data_size") {
          bsize = kv.second.AsInt();
        } else {
          return false;
        }
      }
    }
    tcserve_ref& ref = pr->in[idx];
    if (has_shm) {
      ShmEntry e;
      const int kind = lookup(region, &e);
      if (kind < 0) return fail("Unable to find shared memory region: '" + region + "'");
      if (!ShmRangeOk(roff, rbytes, e.bytes))
        return fail("Invalid offset + byte size for shared memory region: '" + region + "'");
      if (static_cast<uint64_t>(rbytes) < need)
        return fail("input '" + d.name + "' shared memory region is smaller than the tensor");
      ref = tcserve_ref{kind, e.device, e.ptr + roff, need};
      pr->pins.push_back(e.pin);
    } else {
      if (bsize < 0) return false;
      if (static_cast<uint64_t>(bsize) != need) return fail("unexpected byte size for input '" + d.name + "'");
      if (data_off + need > body->size()) return fail("input '" + d.name + "' has no data");
      pr->host_in_off.emplace_back(idx, data_off);
      data_off += need;
      ref = tcserve_ref{0, 0, 0, need};
    }
  }
  const size_t no = m->outputs.size();
  pr->out.assign(no, tcserve_ref{0, 0, 0, 0});
  pr->out_shm.assign(no, false);
  pr->out_region.assign(no, "");
  pr->out_region_bytes.assign(no, 0);
  pr->out_region_offset.assign(no, 0);
  pr->host_out.resize(no);
  const js::Value* outputs = root.Find("outputs");
  pr->out_requested.assign(no, !outputs || outputs->Size() == 0);
  if (!outputs || outputs->Size() == 0) {
    if (!binary_out_default) return false;  // JSON output data: Python server
  } else {
    for (const js::Value& o : outputs->Elements()) {
      const js::Value* nm = o.Find("name");
      if (!nm) return false;
      int idx = -1;
      for (size_t k = 0; k < no; ++k)
        if (m->outputs[k].name == nm->AsString()) idx = static_cast<int>(k);
      if (idx < 0) return false;
      pr->out_requested[idx] = true;
      std::string region;
      int64_t rbytes = 0, roff = 0;
      bool has_shm = false, binary = binary_out_default;
      if (const js::Value* op = o.Find("parameters")) {
        for (const auto& kv : op->Members()) {
          if (kv.first == "shared_memory_region") {
            region = kv.second.AsString();
            has_shm = true;
          } else if (kv.first == "shared_memory_byte_size") {
            rbytes = kv.second.AsInt();
          } else if (kv.first == "shared_memory_offset") {
            roff = kv.second.AsInt();
          } else if (kv.first == "binary_data") {
            binary = kv.second.AsBool();
          } else {
            return false;  // classification
          }
        }
      }
      const uint64_t need = static_cast<uint64_t>(pr->rows) * m->outputs[idx].sample_bytes;
      if (has_shm) {
        ShmEntry e;
        const int kind = lookup(region, &e);
        if (kind < 0) return fail("Unable to find shared memory region: '" + region + "'");
        if (!ShmRangeOk(roff, rbytes, e.bytes))
          return fail("Invalid offset + byte size for shared memory region: '" + region + "'");
        if (static_cast<uint64_t>(rbytes) < need)
          return fail("shared memory size specified with the request for output '" + m->outputs[idx].name + "' (" +
                      std::to_string(rbytes) + " bytes) should be at least " + std::to_string(need) + " bytes");
        pr->out[idx] = tcserve_ref{kind, e.device, e.ptr + roff, need};
        pr->pins.push_back(e.pin);
        pr->out_shm[idx] = true;
        pr->out_region[idx] = region;
        pr->out_region_bytes[idx] = rbytes;
        pr->out_region_offset[idx] = roff;
      } else if (!binary) {
        return false;  // JSON output data: Python server
      }
    }
  }
  for (size_t k = 0; k < no; ++k) {
    if (pr->out_requested[k] && !pr->out_shm[k]) {
      const uint64_t need = static_cast<uint64_t>(pr->rows) * m->outputs[k].sample_bytes;
      pr->host_out[k].resize(need);
      pr->out[k] = tcserve_ref{0, 0, reinterpret_cast<uint64_t>(&pr->host_out[k][0]), need};
    }
  }
  if (!pr->host_in_off.empty()) {
    pr->body = std::move(*body);
    for (const auto& io : pr->host_in_off)
      pr->in[io.first].ptr = reinterpret_cast<uint64_t>(pr->body.data() + io.second);
  }
  n_native++;
  {
    std::lock_guard<std::mutex> lk(m->mu);
    m->q_rows += pr->rows;
    m->q.push_back(std::move(pr));
  }
  m->cv.notify_one();
  return true;
}

std::string Server::HttpInferResponse(NativeModel* m, PendingReq* pr)
{
  std::string js = "{\"model_name\":";
  tc::json::AppendEscapedString(&js, m->name);
  js += ",\"model_version\":";
  tc::json::AppendEscapedString(&js, m->version);
  if (!pr->id.empty()) {
    js += ",\"id\":";
    tc::json::AppendEscapedString(&js, pr->id);
  }
  js += ",\"outputs\":[";
  size_t binary = 0;
  bool first = true;
  for (size_t k = 0; k < m->outputs.size(); ++k) {
    if (!pr->out_requested[k]) continue;
    const TensorDef& d = m->outputs[k];
    js += first ? "{\"name\":" : ",{\"name\":";
    first = false;
    tc::json::AppendEscapedString(&js, d.name);
    js += ",\"datatype\":\"" + d.dtype + "\",\"shape\":[";
    bool fd = true;
    if (m->max_batch > 0) {
      js += std::to_string(pr->rows);
      fd = false;
    }
    for (auto dim : d.dims) {
      js += (fd ? "" : ",") + std::to_string(dim);
      fd = false;
    }
    js += "],\"parameters\":{";
    if (pr->out_shm[k]) {
      js += "\"shared_memory_region\":";
      tc::json::AppendEscapedString(&js, pr->out_region[k]);
      js += ",\"shared_memory_byte_size\":" + std::to_string(pr->out_region_bytes[k]);
      if (pr->out_region_offset[k]) js += ",\"shared_memory_offset\":" + std::to_string(pr->out_region_offset[k]);
    } else {
      js += "\"binary_data_size\":" + std::to_string(pr->host_out[k].size());
      binary += pr->host_out[k].size();
    }
    js += "}}";
  }
  js += "]}";
  std::string r = HttpStatusLine(200);
  if (binary) {
    r += "Content-Type: application/octet-stream\r\nInference-Header-Content-Length: " + std::to_string(js.size()) +
         "\r\n";
  } else {
    r += "Content-Type: application/json\r\n";
  }
  if (pr->http_resp_enc) {
    std::vector<std::pair<const char*, size_t>> parts{{js.data(), js.size()}};
    for (size_t k = 0; k < m->outputs.size(); ++k)
      if (pr->out_requested[k] && !pr->out_shm[k]) parts.emplace_back(pr->host_out[k].data(), pr->host_out[k].size());
    std::string z;
    if (DeflateParts(parts, pr->http_resp_enc, &z)) {
      r += pr->http_resp_enc == 1 ? "Content-Encoding: gzip\r\n" : "Content-Encoding: deflate\r\n";
      r += "Content-Length: " + std::to_string(z.size()) + "\r\n";
      if (pr->http_close) r += "Connection: close\r\n";
      r += "\r\n";
      r += z;
      return r;
    }
  }
  r += "Content-Length: " + std::to_string(js.size() + binary) + "\r\n";
  if (pr->http_close) r += "Connection: close\r\n";
  r += "\r\n";
  r.reserve(r.size() + js.size() + binary);
  r += js;
  for (size_t k = 0; k < m->outputs.size(); ++k)
    if (pr->out_requested[k] && !pr->out_shm[k]) r += pr->host_out[k];
  return r;
}

void Server::FailPending(PendingReq* pr, int grpc_status, int http_status, const std::string& msg)
{
  if (pr->http) PostHttp(pr->loop, pr->conn_id, pr->http_seq, HttpError(http_status, msg, pr->http_close), pr->http_close);
  else PostReply(pr->loop, pr->conn_id, pr->stream_id, std::string(), grpc_status, msg);
}

void Server::PostHttp(Loop* loop, uint64_t conn_id, uint64_t seq, std::string&& bytes, bool close)
{
  auto b = std::make_shared<std::string>(std::move(bytes));
  loop->Post([loop, conn_id, seq, b, close] {
    Conn* c = loop->Find(conn_id);
    if (!c) return;
    c->ready[seq] = std::move(*b);
    for (auto it = c->ready.find(c->resp_seq); it != c->ready.end(); it = c->ready.find(c->resp_seq)) {
      if (c->sendpos == c->sendbuf.size()) {
        c->sendbuf.clear();
        c->sendpos = 0;
      }
      c->sendbuf += it->second;
      c->ready.erase(it);
      c->resp_seq++;
    }
    if (close) c->close_after = true;
    loop->Flush(c);
  });
}

void Server::ProxyHttp(Loop* loop, uint64_t conn_id, uint64_t seq, bool close, std::string&& raw)
{
  n_proxied++;
  proxies_++;
  auto req = std::make_shared<std::string>(std::move(raw));
  std::thread([this, loop, conn_id, seq, close, req] {
    std::string resp;
    std::string e = [&]() -> std::string {
      tc::Socket sock;
      std::string err = sock.Connect(up_http_host_, up_http_port_, 60000000, tc::TlsConfig());
      if (!err.empty()) return err;
      size_t sent = 0;
      while (sent < req->size()) {
        struct iovec iov = {const_cast<char*>(req->data()) + sent, req->size() - sent};
        const ssize_t w = sock.Writev(&iov, 1);
        if (w < 0) return "upstream write failed";
        if (w == 0 && !sock.Wait(true, 60000000)) return "upstream write timed out";
        sent += static_cast<size_t>(w);
      }
      // relay the raw response bytes; the parser only finds where it ends
      tc::HttpResponseParser parser;
      parser.Reset(false);
      char buf[65536];
      while (parser.state() != tc::HttpResponseParser::State::Done) {
        if (parser.state() == tc::HttpResponseParser::State::Error) return "malformed upstream response: " + parser.error();
        const ssize_t n = sock.Read(buf, sizeof(buf));
        if (n == -2) {
          if (!sock.Wait(false, 60000000)) return "upstream read timed out";
          continue;
        }
        if (n <= 0) return resp.empty() ? "upstream closed the connection" : "";
        resp.append(buf, n);
        parser.Feed(buf, static_cast<size_t>(n));
      }
      return "";
    }();
    if (!e.empty()) resp = HttpError(502, "tcserve: upstream HTTP server: " + e, close);
    PostHttp(loop, conn_id, seq, std::move(resp), close);
    proxies_--;
  }).detach();
}

bool Server::ListenHttp(const std::string& host, int port, const std::string& up_host, int up_port, std::string* err)
{
  up_http_host_ = up_host;
  up_http_port_ = up_port;
  int fd = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(port));
  if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) a.sin_addr.s_addr = htonl(INADDR_ANY);
  if (bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || listen(fd, 1024) != 0) {
    *err = "cannot bind/listen on HTTP port " + std::to_string(port) + ": " + strerror(errno);
    close(fd);
    return false;
  }
  socklen_t al = sizeof(a);
  getsockname(fd, reinterpret_cast<sockaddr*>(&a), &al);
  http_port_ = ntohs(a.sin_port);
  loops[0]->http_listen_fd = fd;
  loops[0]->AddListener(fd, 2);
  return true;
}

void Server::OnRequestComplete(Conn* c, Stream* st)
{
  if (st->started) return;
  st->started = true;
  if (st->path == kInferPath) {
    const std::string& in = st->inbuf;
    if (in.size() >= 5 && in[0] == 0) {
      // one uncompressed message: parse it in place (raw tensors are not copied)
      const uint8_t* p = reinterpret_cast<const uint8_t*>(in.data());
      const uint32_t n = (uint32_t(p[1]) << 24) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 8) | p[4];
      if (in.size() == 5 + static_cast<size_t>(n)) {
        if (TryNative(c, st, in.data() + 5, n, &st->inbuf)) return;
        Proxy(c, st, false);  // forward the frame as received
        return;
      }
    }
    std::vector<std::string> msgs;
    std::string err;
    const bool compressed = in.size() >= 5 && in[0] != 0;
    if (!PopMessages(st, &msgs, &err) || msgs.size() != 1) {
      Reply(c, st, nullptr, kInternal, err.empty() ? "expected one request message" : err);
      return;
    }
    if (compressed) n_inflated++;  // a grpc-encoding gzip/deflate message, decompressed here
    if (TryNative(c, st, msgs[0].data(), msgs[0].size(), &msgs[0])) return;
    // not native: forward the (decompressed) message we already popped
    st->inbuf.clear();
    tc::GrpcFrame(msgs[0], tc::GrpcCompression::NONE, &st->inbuf);
  }
  Proxy(c, st, false);
}

void Server::Proxy(Conn* c, Stream* st, bool streaming)
{
  n_proxied++;
  auto ch = Upstream();
  if (!ch) {
    Reply(c, st, nullptr, kUnavailable, "upstream server unavailable");
    return;
  }
  Loop* loop = c->loop;
  const uint64_t cid = c->id;
  const int32_t sid = st->id;
  tc::H2CallHandlers h;
  h.on_message = [this, loop, cid, sid](std::string&& m) {
    auto mm = std::make_shared<std::string>(std::move(m));
    loop->Post([this, loop, cid, sid, mm] {
      Conn* c2 = loop->Find(cid);
      if (!c2) return;
      auto it = c2->streams.find(sid);
      if (it == c2->streams.end()) return;
      Reply(c2, it->second.get(), mm.get(), -1, "");
      loop->Flush(c2);
    });
  };
  h.on_close = [this, loop, cid, sid](const tc::GrpcStatus& s) {
    loop->Post([this, loop, cid, sid, s] {
      Conn* c2 = loop->Find(cid);
      if (!c2) return;
      auto it = c2->streams.find(sid);
      if (it == c2->streams.end()) return;
      it->second->upstream.reset();
      Reply(c2, it->second.get(), nullptr, s.code, s.message);
      loop->Flush(c2);
    });
  };
  st->upstream = ch->StartCall(st->path, st->meta, 0, tc::GrpcCompression::NONE, h);
  if (!st->upstream) {
    Reply(c, st, nullptr, kUnavailable, "upstream call failed");
    return;
  }
  if (!streaming) {
    std::vector<std::string> msgs;
    std::string err;
    if (!PopMessages(st, &msgs, &err)) {
      st->upstream->Cancel();
      return;
    }
    for (auto& m : msgs) st->upstream->Write(std::move(m));
    st->upstream->WritesDone();
  }
}

void Server::OnStreamMessage(Conn* c, Stream* st, std::string&& msg)
{
  if (!st->started) {
    st->started = true;
    Proxy(c, st, true);
  }
  if (!msg.empty() && st->upstream) st->upstream->Write(std::move(msg));
}

void Server::OnStreamEnd(Conn* c, Stream* st)
{
  if (!st->started) {
    st->started = true;
    Proxy(c, st, true);
  }
  if (st->upstream) st->upstream->WritesDone();
}

void Server::OnStreamClosed(Conn*, Stream* st)
{
  if (st->upstream) {
    st->upstream->Cancel();
    st->upstream.reset();
  }
}

// ---------------------------------------------------------------------------
// Native fast path
// ---------------------------------------------------------------------------
NativeModel* Server::FindModel(const std::string& name)
{
  std::lock_guard<std::mutex> lk(models_mu);
  auto it = models.find(name);
  return it == models.end() ? nullptr : it->second.get();
}

// Splits a serialized ModelInferRequest into its small fields (copied to
// `small`) and the byte ranges of its raw_input_contents (field 7), so the
// tensors can be used where they arrived instead of being copied by the parser.
static bool SplitRawInputs(const char* p, size_t n, std::string* small, std::vector<std::pair<size_t, size_t>>* raws)
{
  size_t pos = 0;
  auto varint = [&](uint64_t* v) {
    *v = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      if (pos >= n) return false;
      const uint8_t b = static_cast<uint8_t>(p[pos++]);
      *v |= static_cast<uint64_t>(b & 0x7f) << shift;
      if (!(b & 0x80)) return true;
    }
    return false;
  };
  small->reserve(4096);
  while (pos < n) {
    const size_t start = pos;
    uint64_t tag, v;
    if (!varint(&tag)) return false;
    switch (tag & 7) {
      case 0:
        if (!varint(&v)) return false;
        break;
      case 1:
        pos += 8;
        break;
      case 5:
        pos += 4;
        break;
      case 2:
        if (!varint(&v) || v > n - pos) return false;
        if ((tag >> 3) == 7) {
          raws->emplace_back(pos, static_cast<size_t>(v));
          pos += v;
          continue;
        }
        pos += v;
        break;
      default:
        return false;
    }
    if (pos > n) return false;
    small->append(p + start, pos - start);
  }
  return true;
}

bool Server::TryNative(Conn* c, Stream* st, const char* msg, size_t len, std::string* owner)
{
  inference::ModelInferRequest req;
  std::string small;
  std::vector<std::pair<size_t, size_t>> raws;  // offsets relative to msg
  if (!SplitRawInputs(msg, len, &small, &raws) || !req.ParseFromString(small)) return false;
  const size_t msg_off = static_cast<size_t>(msg - owner->data());
  std::shared_ptr<NativeModel> m;
  {
    std::lock_guard<std::mutex> lk(models_mu);
    auto it = models.find(req.model_name());
    if (it == models.end()) return false;
    m = it->second;
  }
  if (!req.model_version().empty() && req.model_version() != m->version) return false;
  // features the fast path leaves to the Python server
  for (const auto& kv : req.parameters())
    if (kv.first != "triton_enable_empty_final_response" && kv.first != "priority" && kv.first != "timeout")
      return false;
  if (req.inputs_size() != static_cast<int>(m->inputs.size())) return false;
  std::unique_ptr<PendingReq> pr(new PendingReq());
  pr->conn_id = c->id;
  pr->loop = c->loop;
  pr->stream_id = st->id;
  pr->id = req.id();
  pr->t_arrive = NowNs();
  pr->in.resize(m->inputs.size());
  pr->rows = -1;
  int raw_idx = 0;
  auto fail = [&](const std::string& msg) {
    Reply(c, st, nullptr, kInvalidArgument, msg);
    std::lock_guard<std::mutex> lk(m->smu);
    m->fail.count++;
    m->fail.ns += NowNs() - pr->t_arrive;
    return true;
  };
  std::vector<bool> seen(m->inputs.size(), false);
  for (int i = 0; i < req.inputs_size(); ++i) {
    const auto& t = req.inputs(i);
    int idx = -1;
    for (size_t k = 0; k < m->inputs.size(); ++k)
      if (m->inputs[k].name == t.name()) idx = static_cast<int>(k);
    if (idx < 0) return false;
    if (seen[idx]) return fail("input '" + t.name() + "' is specified more than once");
    seen[idx] = true;
    const TensorDef& d = m->inputs[idx];
    if (t.datatype() != d.dtype || t.has_contents()) return false;
    const auto& shape = t.shape();
    if (shape.size() != d.dims.size() + (m->max_batch > 0 ? 1 : 0)) return false;
    int rows = 1;
    size_t off = 0;
    if (m->max_batch > 0) {
      rows = static_cast<int>(shape[0]);
      off = 1;
    }
    for (size_t k = 0; k < d.dims.size(); ++k)
      if (shape[k + off] != d.dims[k]) return false;
    if (rows < 1 || (m->max_batch > 0 && rows > m->max_batch)) return false;
    if (pr->rows >= 0 && pr->rows != rows) return false;
    pr->rows = rows;
    const uint64_t need = static_cast<uint64_t>(rows) * d.sample_bytes;
    std::string region;
    int64_t rbytes = 0, roff = 0;
    bool has_shm = false;
    for (const auto& kv : t.parameters()) {
      if (kv.first == "shared_memory_region") {
        region = kv.second.string_param();
        has_shm = true;
      } else if (kv.first == "shared_memory_byte_size") {
        rbytes = kv.second.int64_param();
      } else if (kv.first == "shared_memory_offset") {
        roff = kv.second.int64_param();
      } else {
        return false;
      }
    }
    tcserve_ref& ref = pr->in[idx];
    if (has_shm) {
      ShmEntry e;
      int kind = -1;
      {
        std::lock_guard<std::mutex> lk(shm_mu_);
        for (int kk = 0; kk < 2 && kind < 0; ++kk) {
          auto it = shm_[kk].find(region);
          if (it != shm_[kk].end()) {
            e = it->second;
            kind = kk;
          }
        }
      }
      if (kind < 0) return fail("Unable to find shared memory region: '" + region + "'");
      if (!ShmRangeOk(roff, rbytes, e.bytes))
        return fail("Invalid offset + byte size for shared memory region: '" + region + "'");
      if (static_cast<uint64_t>(rbytes) < need)
        return fail("input '" + d.name + "' shared memory region is smaller than the tensor");
      ref.kind = kind;
      ref.device = e.device;
      ref.ptr = e.ptr + roff;
      pr->pins.push_back(e.pin);
      ref.bytes = need;
    } else {
      if (raw_idx >= static_cast<int>(raws.size())) return fail("input '" + d.name + "' has no data");
      const auto& rv = raws[raw_idx++];
      if (rv.second != need) return fail("unexpected byte size for input '" + d.name + "'");
      pr->host_in_off.emplace_back(idx, msg_off + rv.first);  // pointer fixed up once the body is owned
      ref.kind = 0;
      ref.device = 0;
      ref.ptr = 0;
      ref.bytes = need;
    }
  }
  // outputs
  const size_t no = m->outputs.size();
  pr->out.assign(no, tcserve_ref{0, 0, 0, 0});
  pr->out_requested.assign(no, req.outputs_size() == 0);
  pr->out_shm.assign(no, false);
  pr->out_region.assign(no, "");
  pr->out_region_bytes.assign(no, 0);
  pr->out_region_offset.assign(no, 0);
  pr->host_out.resize(no);
  for (int i = 0; i < req.outputs_size(); ++i) {
    const auto& o = req.outputs(i);
    int idx = -1;
    for (size_t k = 0; k < no; ++k)
      if (m->outputs[k].name == o.name()) idx = static_cast<int>(k);
    if (idx < 0) return false;
    pr->out_requested[idx] = true;
    std::string region;
    int64_t rbytes = 0, roff = 0;
    bool has_shm = false;
    for (const auto& kv : o.parameters()) {
      if (kv.first == "shared_memory_region") {
        region = kv.second.string_param();
        has_shm = true;
      } else if (kv.first == "shared_memory_byte_size") {
        rbytes = kv.second.int64_param();
      } else if (kv.first == "shared_memory_offset") {
        roff = kv.second.int64_param();
      } else if (kv.first == "binary_data") {
      } else {
        return false;  // classification etc.
      }
    }
    const uint64_t need = static_cast<uint64_t>(pr->rows) * m->outputs[idx].sample_bytes;
    if (has_shm) {
      ShmEntry e;
      int kind = -1;
      {
        std::lock_guard<std::mutex> lk(shm_mu_);
        for (int kk = 0; kk < 2 && kind < 0; ++kk) {
          auto it = shm_[kk].find(region);
          if (it != shm_[kk].end()) {
            e = it->second;
            kind = kk;
          }
        }
      }
      if (kind < 0) return fail("Unable to find shared memory region: '" + region + "'");
      if (!ShmRangeOk(roff, rbytes, e.bytes))
        return fail("Invalid offset + byte size for shared memory region: '" + region + "'");
      if (static_cast<uint64_t>(rbytes) < need)
        return fail("shared memory size specified with the request for output '" + m->outputs[idx].name + "' (" +
                    std::to_string(rbytes) + " bytes) should be at least " + std::to_string(need) + " bytes");
      pr->out[idx] = tcserve_ref{kind, e.device, e.ptr + roff, need};
      pr->pins.push_back(e.pin);
      pr->out_shm[idx] = true;
      pr->out_region[idx] = region;
      pr->out_region_bytes[idx] = rbytes;
      pr->out_region_offset[idx] = roff;
    }
  }
  for (size_t k = 0; k < no; ++k) {
    if (pr->out_requested[k] && !pr->out_shm[k]) {
      const uint64_t need = static_cast<uint64_t>(pr->rows) * m->outputs[k].sample_bytes;
      pr->host_out[k].resize(need);
      pr->out[k] = tcserve_ref{0, 0, reinterpret_cast<uint64_t>(&pr->host_out[k][0]), need};
    }
  }
  if (!pr->host_in_off.empty()) {
    pr->body = std::move(*owner);  // the heap buffer moves with the string: offsets stay valid
    for (const auto& io : pr->host_in_off)
      pr->in[io.first].ptr = reinterpret_cast<uint64_t>(pr->body.data() + io.second);
  }
  n_native++;
  {
    std::lock_guard<std::mutex> lk(m->mu);
    m->q_rows += pr->rows;
    m->q.push_back(std::move(pr));
  }
  m->cv.notify_one();
  return true;
}

void Server::Worker(std::shared_ptr<NativeModel> m, int instance)
{
  pthread_setname_np(pthread_self(), ("tcs-w" + std::to_string(instance) + "-" + m->name).substr(0, 15).c_str());
  while (true) {
    std::vector<std::unique_ptr<PendingReq>> batch;
    {
      std::unique_lock<std::mutex> lk(m->mu);
      m->cv.wait(lk, [&] { return m->stopping || !m->q.empty(); });
      if (m->stopping) return;
      // dispatch policy (batch_policy.h): re-evaluated after every wake-up
      // until it says go.  The rules and their measured effects:
      //   * pipelined dispatch (per model, opt-in): densenet_onnx bs1 at
      //     concurrency 64 on 2 instances: 18.0-18.4k -> 19.9-22.1k infer/s, p50
      //     3.3 -> 2.4 ms; its headline's full batches never reach this rule.
      //     Off for bert_large, where it locked concurrency 16 into small
      //     batches (profiles/r3_instances.md);
      //   * staggered dispatch of full batches (TCSERVE_STAGGER=0: off):
      //     densenet_onnx headline, 2 instances: p99 9.1-12.2 ms -> 9.1-9.2 ms
      //     on three runs each, same or higher throughput (r3_instances.md).
      static const bool stagger = [] {
        const char* e = getenv("TCSERVE_STAGGER");
        return !e || atoi(e) != 0;
      }();
      tcserve::BatchPolicyConfig pc;
      pc.max_batch = m->max_batch;
      pc.delay_ns = m->delay_ns;
      pc.preferred = m->preferred;
      pc.idle_dispatch = m->idle_dispatch;
      pc.pipelined = m->pipelined;
      pc.stagger = stagger;
      pc.instances = m->instances;
      bool go = false;
      while (!m->stopping && !m->q.empty()) {
        tcserve::BatchPolicyState st;
        st.now_ns = NowNs();
        st.front_arrive_ns = m->q.front()->t_arrive;
        st.q_rows = m->q_rows;
        st.busy = m->busy;
        st.last_rows = m->last_rows;
        st.ema_exec_ns = m->ema_exec_ns;
        st.last_start_ns = m->last_start_ns;
        const uint64_t until = tcserve::WaitUntil(pc, st);
        if (!until) {
          go = true;
          break;
        }
        m->cv.wait_for(lk, std::chrono::nanoseconds(until - st.now_ns));
      }
      if (m->stopping) return;
      if (!go) continue;  // another worker emptied the queue
      m->last_start_ns = NowNs();
      const int limit = tcserve::TakeLimit(pc, m->q_rows);
      int rows = 0;
      while (!m->q.empty() && (rows == 0 || rows + m->q.front()->rows <= limit)) {
        rows += m->q.front()->rows;
        m->q_rows -= m->q.front()->rows;
        batch.push_back(std::move(m->q.front()));
        m->q.pop_front();
      }
      if (!m->q.empty()) m->cv.notify_one();
      m->last_rows = rows;
      m->busy++;
    }
    const uint64_t t_exec = NowNs();
    Execute(m, instance, batch);
    const double d_exec = static_cast<double>(NowNs() - t_exec);
    {
      std::lock_guard<std::mutex> lk(m->mu);
      m->busy--;
      m->ema_exec_ns = m->ema_exec_ns > 0 ? 0.9 * m->ema_exec_ns + 0.1 * d_exec : d_exec;
    }
    m->cv.notify_all();  // a worker holding a partial batch may dispatch now
  }
}

void Server::Execute(const std::shared_ptr<NativeModel>& ms, int instance,
                     std::vector<std::unique_ptr<PendingReq>>& batch)
{
  NativeModel* m = ms.get();
  const int n = static_cast<int>(batch.size());
  const size_t ni = m->inputs.size(), no = m->outputs.size();
  std::vector<int32_t> rows(n);
  std::vector<tcserve_ref> ins(n * ni), outs(n * no);
  int total = 0;
  for (int r = 0; r < n; ++r) {
    rows[r] = batch[r]->rows;
    total += rows[r];
    for (size_t k = 0; k < ni; ++k) ins[r * ni + k] = batch[r]->in[k];
    for (size_t k = 0; k < no; ++k) outs[r * no + k] = batch[r]->out[k];
  }
  uint64_t timing[3] = {0, 0, 0};
  tcserve_batch b;
  b.n_requests = n;
  b.total_rows = total;
  b.rows = rows.data();
  b.n_inputs = static_cast<int32_t>(ni);
  b.inputs = ins.data();
  b.n_outputs = static_cast<int32_t>(no);
  b.outputs = outs.data();
  b.timing_ns = timing;
  char err[1024] = {0};
  const uint64_t t_exec = NowNs();
  int rc;
  {
    char tag[160];
    snprintf(tag, sizeof(tag), "tcserve.batch %s inst=%d requests=%d rows=%d", m->name.c_str(), instance, n, total);
    triton::client::trace::Range range(tag);
    rc = m->fn(m->user, instance, &b, err, sizeof(err));
  }
  const uint64_t t_done = NowNs();
  {
    std::lock_guard<std::mutex> lk(m->smu);
    if (rc == 0) {
      m->execution_count++;
      m->inference_count += total;
      BatchStat& bs = m->batch[total];
      bs.count++;
      bs.in_ns += timing[0];
      bs.infer_ns += timing[1];
      bs.out_ns += timing[2];
      m->cin.count += n;
      m->cin.ns += timing[0];
      m->cinf.count += n;
      m->cinf.ns += timing[1];
      m->cout.count += n;
      m->cout.ns += timing[2];
    }
    m->last_inference_ms =
        std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::system_clock::now().time_since_epoch())
            .count();
    for (auto& pr : batch) {
      Stat& s = rc == 0 ? m->success : m->fail;
      s.count++;
      s.ns += t_done - pr->t_arrive;
      if (rc == 0) {
        m->queue.count++;
        m->queue.ns += t_exec - pr->t_arrive;
      }
    }
  }
  for (auto& pr : batch) {
    if (rc != 0) {
      FailPending(pr.get(), kInternal, 500, err);
      continue;
    }
    if (pr->http) {
      if (pr->http_resp_enc) {
        // compressed response: built and deflated on the codec pool (the
        // request, its host outputs and the model stay alive with the task)
        n_deflated++;
        std::shared_ptr<PendingReq> own(pr.release());
        std::shared_ptr<NativeModel> keep = ms;
        codec_.Submit([this, own, keep] {
          PostHttp(own->loop, own->conn_id, own->http_seq, HttpInferResponse(keep.get(), own.get()), own->http_close);
        });
        continue;
      }
      PostHttp(pr->loop, pr->conn_id, pr->http_seq, HttpInferResponse(m, pr.get()), pr->http_close);
      continue;
    }
    inference::ModelInferResponse resp;
    resp.set_model_name(m->name);
    resp.set_model_version(m->version);
    resp.set_id(pr->id);
    int last_raw = -1;
    std::vector<int> order;
    for (size_t k = 0; k < no; ++k)
      if (pr->out_requested[k]) order.push_back(static_cast<int>(k));
    for (size_t j = 0; j < order.size(); ++j) {
      const int k = order[j];
      auto* o = resp.add_outputs();
      o->set_name(m->outputs[k].name);
      o->set_datatype(m->outputs[k].dtype);
      if (m->max_batch > 0) o->add_shape(pr->rows);
      for (auto d : m->outputs[k].dims) o->add_shape(d);
      if (pr->out_shm[k]) {
        (*o->mutable_parameters())["shared_memory_region"].set_string_param(pr->out_region[k]);
        (*o->mutable_parameters())["shared_memory_byte_size"].set_int64_param(pr->out_region_bytes[k]);
        if (pr->out_region_offset[k])
          (*o->mutable_parameters())["shared_memory_offset"].set_int64_param(pr->out_region_offset[k]);
      } else {
        last_raw = static_cast<int>(j);
      }
    }
    // raw_output_contents stays position-aligned with outputs (empty for shm outputs)
    for (int j = 0; j <= last_raw; ++j) {
      const int k = order[j];
      std::string* dst = resp.add_raw_output_contents();
      if (!pr->out_shm[k]) *dst = std::move(pr->host_out[k]);
    }
    std::string enc;
    resp.Encode(&enc);
    PostReply(pr->loop, pr->conn_id, pr->stream_id, std::move(enc), kOk, "");
  }
}

int Server::AddModel(std::unique_ptr<NativeModel> m, std::string* err)
{
  std::shared_ptr<NativeModel> sm(m.release());
  std::lock_guard<std::mutex> lk(models_mu);
  if (models.count(sm->name)) {
    *err = "model '" + sm->name + "' already registered";
    return 1;
  }
  for (int i = 0; i < std::max(1, sm->instances); ++i)
    sm->workers.emplace_back(&Server::Worker, this, sm, i);
  models[sm->name] = sm;
  return 0;
}

int Server::RemoveModel(const std::string& name)
{
  std::shared_ptr<NativeModel> m;
  {
    std::lock_guard<std::mutex> lk(models_mu);
    auto it = models.find(name);
    if (it == models.end()) return 1;
    m = it->second;
    models.erase(it);
  }
  {
    std::lock_guard<std::mutex> lk(m->mu);
    m->stopping = true;
  }
  m->cv.notify_all();
  for (auto& t : m->workers)
    if (t.joinable()) t.join();
  // fail what was still queued
  for (auto& pr : m->q) FailPending(pr.get(), kUnavailable, 503, "model unloaded");
  m->q.clear();
  return 0;
}

void Server::ShmAdd(int kind, const std::string& name, const ShmEntry& e)
{
  std::lock_guard<std::mutex> lk(shm_mu_);
  shm_[kind][name] = e;
}

int Server::ShmRemove(int kind, const std::string& name)
{
  // Take the entries out of the map (no new request can pin them).  Requests
  // already queued or executing keep their pins; the entry moves to the
  // draining list and the caller must not unmap / hipIpcCloseMemHandle the
  // region until ShmBusy() says the last pin has dropped.  Never blocks.
  std::lock_guard<std::mutex> lk(shm_mu_);
  std::vector<std::pair<std::string, ShmEntry>> gone;
  if (name.empty()) {
    for (auto& kv : shm_[kind]) gone.emplace_back(kv.first, kv.second);
    shm_[kind].clear();
  } else {
    auto it = shm_[kind].find(name);
    if (it != shm_[kind].end()) {
      gone.emplace_back(it->first, it->second);
      shm_[kind].erase(it);
    }
  }
  int busy = 0;
  for (auto& g : gone) {
    if (g.second.pin.use_count() > 1) {
      draining_.push_back(Draining{kind, g.second.ptr, g.second.pin});
      ++busy;
    }
  }
  return busy;
}

int Server::ShmBusy(int kind, uint64_t ptr)
{
  std::lock_guard<std::mutex> lk(shm_mu_);
  draining_.erase(std::remove_if(draining_.begin(), draining_.end(),
                                 [](const Draining& d) { return d.pin.use_count() <= 1; }),
                  draining_.end());
  for (const auto& d : draining_)
    if (d.kind == kind && d.ptr == ptr) return 1;
  return 0;
}

}  // namespace tcserve

// ===========================================================================
// C ABI
// ===========================================================================
using tcserve::NativeModel;
using tcserve::Server;

static void SetErr(char* err, int32_t errlen, const std::string& m)
{
  if (err && errlen > 0) {
    strncpy(err, m.c_str(), errlen - 1);
    err[errlen - 1] = 0;
  }
}

extern "C" {

void* tcserve_create(const char* host, int32_t port, const char* upstream_host, int32_t upstream_port,
                     int32_t io_threads, char* err, int32_t errlen)
{
  std::unique_ptr<Server> s(new Server());
  std::string e;
  if (!s->Start(host ? host : "0.0.0.0", port, upstream_host ? upstream_host : "127.0.0.1", upstream_port,
                io_threads, &e)) {
    SetErr(err, errlen, e);
    return nullptr;
  }
  return s.release();
}

int32_t tcserve_port(void* server) { return static_cast<Server*>(server)->port(); }

int32_t tcserve_listen_http(void* server, const char* host, int32_t port, const char* upstream_host,
                            int32_t upstream_port, char* err, int32_t errlen)
{
  std::string e;
  Server* s = static_cast<Server*>(server);
  if (!s->ListenHttp(host ? host : "0.0.0.0", port, upstream_host ? upstream_host : "127.0.0.1", upstream_port, &e)) {
    SetErr(err, errlen, e);
    return -1;
  }
  return s->http_port();
}

int32_t tcserve_add_model(void* server, const char* name, const char* version, int32_t max_batch,
                          int32_t max_queue_delay_us, int32_t instances, int32_t n_inputs, const char** in_names,
                          const char** in_dtypes, const int32_t* in_ndims, const int64_t* in_dims, int32_t n_outputs,
                          const char** out_names, const char** out_dtypes, const int32_t* out_ndims,
                          const int64_t* out_dims, tcserve_exec_fn fn, void* user, char* err, int32_t errlen)
{
  std::unique_ptr<NativeModel> m(new NativeModel());
  m->name = name;
  m->version = version;
  m->max_batch = max_batch;
  m->delay_ns = static_cast<uint64_t>(std::max(0, max_queue_delay_us)) * 1000ull;
  m->instances = instances;
  m->fn = fn;
  m->user = user;
  auto fill = [&](int32_t n, const char** names, const char** dts, const int32_t* nd, const int64_t* dims,
                  std::vector<tcserve::TensorDef>* out) -> bool {
    size_t p = 0;
    for (int i = 0; i < n; ++i) {
      tcserve::TensorDef d;
      d.name = names[i];
      d.dtype = dts[i];
      size_t elems = 1;
      for (int k = 0; k < nd[i]; ++k) {
        d.dims.push_back(dims[p]);
        if (dims[p] < 0) return false;
        elems *= static_cast<size_t>(dims[p]);
        ++p;
      }
      const size_t es = tcserve::DtypeSize(d.dtype);
      if (es == 0) return false;
      d.sample_bytes = elems * es;
      out->push_back(d);
    }
    return true;
  };
  if (!fill(n_inputs, in_names, in_dtypes, in_ndims, in_dims, &m->inputs) ||
      !fill(n_outputs, out_names, out_dtypes, out_ndims, out_dims, &m->outputs)) {
    SetErr(err, errlen, "native models need fixed-size, fixed-width tensors");
    return 1;
  }
  std::string e;
  if (static_cast<Server*>(server)->AddModel(std::move(m), &e) != 0) {
    SetErr(err, errlen, e);
    return 1;
  }
  return 0;
}

int32_t tcserve_remove_model(void* server, const char* name) { return static_cast<Server*>(server)->RemoveModel(name); }

int32_t tcserve_set_idle_dispatch(void* server, const char* name, int32_t on)
{
  Server* s = static_cast<Server*>(server);
  std::shared_ptr<NativeModel> m;
  {
    std::lock_guard<std::mutex> lk(s->models_mu);
    auto it = s->models.find(name);
    if (it == s->models.end()) return 1;
    m = it->second;
  }
  std::lock_guard<std::mutex> lk(m->mu);
  m->idle_dispatch = (on & 1) != 0;  // bit 0: idle-aware dispatch
  m->pipelined = (on & 2) != 0;      // bit 1: pipelined dispatch of partial batches
  return 0;
}

int32_t tcserve_batch_policy_sim(int32_t max_batch, uint64_t delay_ns, const int32_t* preferred, int32_t n_pref,
                                 int32_t instances, int32_t flags, const uint64_t* arrive_ns, const int32_t* rows,
                                 int32_t n, uint64_t exec_base_ns, uint64_t exec_per_row_ns, uint64_t* out_start_ns,
                                 int32_t* out_rows, int32_t* out_first, int32_t* out_instance, int32_t max_batches)
{
  if (instances < 1 || n < 0 || n_pref < 0 || (n && (!arrive_ns || !rows)) || (n_pref && !preferred)) return -1;
  tcserve::BatchPolicyConfig pc;
  pc.max_batch = max_batch;
  pc.delay_ns = delay_ns;
  for (int32_t i = 0; i < n_pref; ++i)
    if (preferred[i] > 0) pc.preferred.push_back(preferred[i]);
  std::sort(pc.preferred.begin(), pc.preferred.end());
  pc.idle_dispatch = flags & 1;
  pc.pipelined = (flags & 2) != 0;
  pc.stagger = (flags & 4) != 0;
  pc.instances = instances;
  const int cap = pc.Cap();
  for (int32_t i = 0; i < n; ++i)
    if (rows[i] < 1 || rows[i] > cap || (i && arrive_ns[i] < arrive_ns[i - 1])) return -1;
  std::deque<int32_t> q;
  int q_rows = 0, busy = 0, last_rows = 0, nb = 0;
  double ema = 0;
  uint64_t last_start = 0, t = n ? arrive_ns[0] : 0;
  std::vector<uint64_t> free_at(instances, 0);  // 0 = idle
  std::vector<uint64_t> started(instances, 0);
  int32_t next = 0, done = 0;
  while (done < n) {
    // completions at or before t, then arrivals at or before t
    for (int i = 0; i < instances; ++i)
      if (free_at[i] && free_at[i] <= t) {
        const double d = static_cast<double>(free_at[i] - started[i]);
        ema = ema > 0 ? 0.9 * ema + 0.1 * d : d;
        free_at[i] = 0;
        busy--;
      }
    while (next < n && arrive_ns[next] <= t) {
      q.push_back(next);
      q_rows += rows[next++];
    }
    uint64_t timer = UINT64_MAX;
    while (!q.empty()) {
      int idle = -1;
      for (int i = 0; i < instances && idle < 0; ++i)
        if (!free_at[i]) idle = i;
      if (idle < 0) break;
      tcserve::BatchPolicyState st;
      st.now_ns = t;
      st.front_arrive_ns = arrive_ns[q.front()];
      st.q_rows = q_rows;
      st.busy = busy;
      st.last_rows = last_rows;
      st.ema_exec_ns = ema;
      st.last_start_ns = last_start;
      const uint64_t until = tcserve::WaitUntil(pc, st);
      if (until) {
        timer = until;
        break;
      }
      const int limit = tcserve::TakeLimit(pc, q_rows);
      int r = 0;
      const int32_t first = q.front();
      while (!q.empty() && (r == 0 || r + rows[q.front()] <= limit)) {
        r += rows[q.front()];
        q_rows -= rows[q.front()];
        q.pop_front();
        done++;
      }
      if (nb >= max_batches) return -2;
      out_start_ns[nb] = t;
      out_rows[nb] = r;
      out_first[nb] = first;
      out_instance[nb] = idle;
      nb++;
      last_rows = r;
      last_start = t;
      started[idle] = t;
      free_at[idle] = t + exec_base_ns + exec_per_row_ns * static_cast<uint64_t>(r);
      busy++;
    }
    if (done >= n) break;
    uint64_t nt = timer;
    if (next < n) nt = std::min(nt, arrive_ns[next]);
    for (int i = 0; i < instances; ++i)
      if (free_at[i]) nt = std::min(nt, free_at[i]);
    if (nt == UINT64_MAX) return -1;  // cannot happen: a queued request always has a deadline or a free instance
    t = std::max(t, nt);
  }
  return nb;
}

int32_t tcserve_batch_policy_sim_closed(int32_t max_batch, uint64_t delay_ns, const int32_t* preferred,
                                        int32_t n_pref, int32_t instances, int32_t flags, int32_t clients,
                                        int32_t rows_per_req, uint64_t spread_ns, uint64_t turnaround_ns,
                                        uint64_t resp_spacing_ns, uint64_t exec_base_ns, uint64_t exec_per_row_ns,
                                        uint64_t horizon_ns, uint64_t* out_start_ns, int32_t* out_rows,
                                        int32_t* out_instance, int32_t max_batches)
{
  if (instances < 1 || clients < 1 || n_pref < 0 || (n_pref && !preferred) || !out_start_ns || !out_rows ||
      !out_instance)
    return -1;
  tcserve::BatchPolicyConfig pc;
  pc.max_batch = max_batch;
  pc.delay_ns = delay_ns;
  for (int32_t i = 0; i < n_pref; ++i)
    if (preferred[i] > 0) pc.preferred.push_back(preferred[i]);
  std::sort(pc.preferred.begin(), pc.preferred.end());
  pc.idle_dispatch = flags & 1;
  pc.pipelined = (flags & 2) != 0;
  pc.stagger = (flags & 4) != 0;
  pc.instances = instances;
  if (rows_per_req < 1 || rows_per_req > pc.Cap()) return -1;
  // (arrival time, client), earliest first
  using Ev = std::pair<uint64_t, int32_t>;
  std::priority_queue<Ev, std::vector<Ev>, std::greater<Ev>> arrivals;
  for (int32_t k = 0; k < clients; ++k) arrivals.push({spread_ns * static_cast<uint64_t>(k), k});
  std::deque<int32_t> q;
  std::vector<uint64_t> free_at(instances, 0), started(instances, 0);
  std::vector<std::vector<int32_t>> members(instances);
  std::vector<uint64_t> arrived(clients, 0);
  int q_rows = 0, busy = 0, last_rows = 0, nb = 0;
  double ema = 0;
  uint64_t last_start = 0, t = 0;
  while (true) {
    for (int i = 0; i < instances; ++i)
      if (free_at[i] && free_at[i] <= t) {
        const double d = static_cast<double>(free_at[i] - started[i]);
        ema = ema > 0 ? 0.9 * ema + 0.1 * d : d;
        busy--;
        for (size_t j = 0; j < members[i].size(); ++j)
          arrivals.push({free_at[i] + turnaround_ns + resp_spacing_ns * j, members[i][j]});
        members[i].clear();
        free_at[i] = 0;
      }
    while (!arrivals.empty() && arrivals.top().first <= t) {
      arrived[arrivals.top().second] = arrivals.top().first;
      q.push_back(arrivals.top().second);
      q_rows += rows_per_req;
      arrivals.pop();
    }
    if (t >= horizon_ns) break;
    uint64_t timer = UINT64_MAX;
    while (!q.empty()) {
      int idle = -1;
      for (int i = 0; i < instances && idle < 0; ++i)
        if (!free_at[i]) idle = i;
      if (idle < 0) break;
      tcserve::BatchPolicyState st;
      st.now_ns = t;
      st.q_rows = q_rows;
      st.busy = busy;
      st.last_rows = last_rows;
      st.ema_exec_ns = ema;
      st.last_start_ns = last_start;
      st.front_arrive_ns = arrived[q.front()];
      const uint64_t until = tcserve::WaitUntil(pc, st);
      if (until) {
        timer = until;
        break;
      }
      const int limit = tcserve::TakeLimit(pc, q_rows);
      int r = 0;
      while (!q.empty() && (r == 0 || r + rows_per_req <= limit)) {
        r += rows_per_req;
        q_rows -= rows_per_req;
        members[idle].push_back(q.front());
        q.pop_front();
      }
      if (nb >= max_batches) return -2;
      out_start_ns[nb] = t;
      out_rows[nb] = r;
      out_instance[nb] = idle;
      nb++;
      last_rows = r;
      last_start = t;
      started[idle] = t;
      free_at[idle] = t + exec_base_ns + exec_per_row_ns * static_cast<uint64_t>(r);
      busy++;
    }
    uint64_t nt = std::min(timer, horizon_ns);
    if (!arrivals.empty()) nt = std::min(nt, arrivals.top().first);
    for (int i = 0; i < instances; ++i)
      if (free_at[i]) nt = std::min(nt, free_at[i]);
    t = std::max(t, nt);
  }
  return nb;
}

int32_t tcserve_set_preferred(void* server, const char* name, const int32_t* sizes, int32_t n)
{
  Server* s = static_cast<Server*>(server);
  std::shared_ptr<NativeModel> m;
  {
    std::lock_guard<std::mutex> lk(s->models_mu);
    auto it = s->models.find(name);
    if (it == s->models.end()) return 1;
    m = it->second;
  }
  std::vector<int> v;
  for (int32_t i = 0; i < n; ++i)
    if (sizes[i] > 0) v.push_back(sizes[i]);
  std::sort(v.begin(), v.end());
  std::lock_guard<std::mutex> lk(m->mu);
  m->preferred = std::move(v);
  return 0;
}

int32_t tcserve_shm_add(void* server, const char* name, int32_t kind, uint64_t ptr, uint64_t bytes, int32_t device)
{
  if (kind != 0 && kind != 1) return 1;
  tcserve::ShmEntry e;
  e.ptr = ptr;
  e.bytes = bytes;
  e.device = device;
  static_cast<Server*>(server)->ShmAdd(kind, name, e);
  return 0;
}

int32_t tcserve_shm_remove(void* server, int32_t kind, const char* name)
{
  if (kind != 0 && kind != 1) return -1;
  return static_cast<Server*>(server)->ShmRemove(kind, name ? name : "");
}

int32_t tcserve_shm_busy(void* server, int32_t kind, uint64_t ptr)
{
  if (kind != 0 && kind != 1) return 0;
  return static_cast<Server*>(server)->ShmBusy(kind, ptr);
}

int32_t tcserve_model_stats(void* server, const char* name, uint64_t* out)
{
  Server* s = static_cast<Server*>(server);
  std::shared_ptr<NativeModel> m;
  {
    std::lock_guard<std::mutex> lk(s->models_mu);
    auto it = s->models.find(name);
    if (it == s->models.end()) return 1;
    m = it->second;
  }
  std::lock_guard<std::mutex> lk(m->smu);
  const uint64_t v[11] = {m->inference_count, m->execution_count, m->success.count, m->success.ns, m->fail.count,
                          m->fail.ns, m->queue.ns, m->cin.ns, m->cinf.ns, m->cout.ns, m->last_inference_ms};
  memcpy(out, v, sizeof(v));
  return 0;
}

int32_t tcserve_batch_stats(void* server, const char* name, uint64_t* out, int32_t max_rows)
{
  Server* s = static_cast<Server*>(server);
  std::shared_ptr<NativeModel> m;
  {
    std::lock_guard<std::mutex> lk(s->models_mu);
    auto it = s->models.find(name);
    if (it == s->models.end()) return -1;
    m = it->second;
  }
  std::lock_guard<std::mutex> lk(m->smu);
  int32_t r = 0;
  for (const auto& kv : m->batch) {
    if (r >= max_rows) break;
    uint64_t* row = out + 7 * r;
    row[0] = kv.first;
    row[1] = kv.second.count;
    row[2] = kv.second.in_ns;
    row[3] = kv.second.infer_ns;
    row[4] = kv.second.out_ns;
    row[5] = row[6] = 0;
    ++r;
  }
  return r;
}

int32_t tcserve_counters(void* server, uint64_t* out)
{
  Server* s = static_cast<Server*>(server);
  out[0] = s->n_native.load();
  out[1] = s->n_proxied.load();
  out[2] = s->n_conns.load();
  out[3] = s->n_inflated.load();
  out[4] = s->n_deflated.load();
  return 0;
}

void tcserve_destroy(void* server) { delete static_cast<Server*>(server); }

}  // extern "C"

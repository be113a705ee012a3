// gRPC-over-HTTP/2 channel on nghttp2 (see h2.h).
#include "h2.h"

#include <nghttp2/nghttp2.h>
#include <poll.h>
#include <sys/eventfd.h>
#include <unistd.h>
#include <zlib.h>

#include <cstring>

namespace triton { namespace client {

namespace {

uint64_t
NowNs()
{
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

std::string
PercentDecode(const std::string& s)
{
  std::string out;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size()) {
      out.push_back(static_cast<char>(std::strtol(s.substr(i + 1, 2).c_str(), nullptr, 16)));
      i += 2;
    } else {
      out.push_back(s[i]);
    }
  }
  return out;
}

nghttp2_session*
S(void* p)
{
  return static_cast<nghttp2_session*>(p);
}

int
cb_frame_recv(nghttp2_session*, const nghttp2_frame* frame, void* user)
{
  auto* ch = static_cast<H2Channel*>(user);
  if (frame->hd.type == NGHTTP2_PING && (frame->hd.flags & NGHTTP2_FLAG_ACK)) ch->OnPingAck();
  if (frame->hd.type == NGHTTP2_HEADERS || frame->hd.type == NGHTTP2_DATA) {
    ch->OnFrameRecv(frame->hd.stream_id, (frame->hd.flags & NGHTTP2_FLAG_END_STREAM) != 0,
                    frame->hd.type == NGHTTP2_HEADERS);
  }
  return 0;
}

int
cb_data_chunk(nghttp2_session*, uint8_t, int32_t stream_id, const uint8_t* data, size_t len, void* user)
{
  static_cast<H2Channel*>(user)->OnData(stream_id, data, len);
  return 0;
}

int
cb_stream_close(nghttp2_session*, int32_t stream_id, uint32_t error_code, void* user)
{
  static_cast<H2Channel*>(user)->OnStreamClose(stream_id, error_code);
  return 0;
}

int
cb_header(nghttp2_session*, const nghttp2_frame* frame, const uint8_t* name, size_t namelen, const uint8_t* value,
          size_t valuelen, uint8_t, void* user)
{
  static_cast<H2Channel*>(user)->OnHeader(
      frame->hd.stream_id, std::string(reinterpret_cast<const char*>(name), namelen),
      std::string(reinterpret_cast<const char*>(value), valuelen));
  return 0;
}

ssize_t
cb_read_body(nghttp2_session*, int32_t stream_id, uint8_t* buf, size_t length, uint32_t* data_flags,
             nghttp2_data_source* source, void*)
{
  return static_cast<H2Channel*>(source->ptr)->ReadBody(stream_id, buf, length, data_flags);
}

bool
Inflate(const char* p, size_t n, std::string* out)
{
  z_stream s;
  std::memset(&s, 0, sizeof(s));
  if (inflateInit2(&s, 15 | 32) != Z_OK) return false;
  s.next_in = reinterpret_cast<Bytef*>(const_cast<char*>(p));
  s.avail_in = static_cast<uInt>(n);
  char buf[1 << 16];
  int rc;
  out->clear();
  do {
    s.next_out = reinterpret_cast<Bytef*>(buf);
    s.avail_out = sizeof(buf);
    rc = inflate(&s, Z_NO_FLUSH);
    if (rc != Z_OK && rc != Z_STREAM_END) {
      inflateEnd(&s);
      return false;
    }
    out->append(buf, sizeof(buf) - s.avail_out);
  } while (rc != Z_STREAM_END && s.avail_in > 0);
  inflateEnd(&s);
  return true;
}

}  // namespace

std::string
GrpcStatus::CodeName() const
{
  static const char* names[] = {"OK", "CANCELLED", "UNKNOWN", "INVALID_ARGUMENT", "DEADLINE_EXCEEDED", "NOT_FOUND",
                                "ALREADY_EXISTS", "PERMISSION_DENIED", "RESOURCE_EXHAUSTED", "FAILED_PRECONDITION",
                                "ABORTED", "OUT_OF_RANGE", "UNIMPLEMENTED", "INTERNAL", "UNAVAILABLE", "DATA_LOSS",
                                "UNAUTHENTICATED"};
  return (code >= 0 && code <= 16) ? names[code] : "UNKNOWN";
}

bool
GrpcFrame(const std::string& message, GrpcCompression comp, std::string* out)
{
  std::string payload;
  const std::string* body = &message;
  uint8_t flag = 0;
  if (comp != GrpcCompression::NONE) {
    if (!Compress({{message.data(), message.size()}}, comp == GrpcCompression::GZIP, &payload)) return false;
    body = &payload;
    flag = 1;
  }
  uint32_t n = static_cast<uint32_t>(body->size());
  out->clear();
  out->reserve(5 + n);
  out->push_back(static_cast<char>(flag));
  out->push_back(static_cast<char>((n >> 24) & 0xff));
  out->push_back(static_cast<char>((n >> 16) & 0xff));
  out->push_back(static_cast<char>((n >> 8) & 0xff));
  out->push_back(static_cast<char>(n & 0xff));
  out->append(*body);
  return true;
}

//==============================================================================
std::shared_ptr<H2Channel>
H2Channel::Create(const std::string& host, int port, const H2ChannelOptions& opts, std::string* err)
{
  // The last owner may be released ON the io thread (a finished call or a
  // posted task holding the channel): joining there would be a self-join
  // (EDEADLK -> std::terminate), so that case only flags the loop, which
  // exits and deletes the channel itself.
  std::shared_ptr<H2Channel> ch(new H2Channel(), [](H2Channel* p) {
    if (p->io_.joinable() && p->io_.get_id() == std::this_thread::get_id()) {
      p->delete_on_exit_ = true;
      p->stop_ = true;
      return;
    }
    delete p;
  });
  ch->opts_ = opts;
  ch->authority_ = host + ":" + std::to_string(port);
  std::string e = ch->sock_.Connect(host, port, 20000000, opts.tls);
  if (!e.empty()) {
    *err = e;
    return nullptr;
  }
  ch->sock_.SetNonBlocking(true);
  nghttp2_session_callbacks* cbs;
  nghttp2_session_callbacks_new(&cbs);
  nghttp2_session_callbacks_set_on_frame_recv_callback(cbs, cb_frame_recv);
  nghttp2_session_callbacks_set_on_data_chunk_recv_callback(cbs, cb_data_chunk);
  nghttp2_session_callbacks_set_on_stream_close_callback(cbs, cb_stream_close);
  nghttp2_session_callbacks_set_on_header_callback(cbs, cb_header);
  nghttp2_session* session;
  nghttp2_option* option;
  nghttp2_option_new(&option);
  nghttp2_option_set_peer_max_concurrent_streams(option, 1u << 20);
  int rc = nghttp2_session_client_new2(&session, cbs, ch.get(), option);
  nghttp2_option_del(option);
  nghttp2_session_callbacks_del(cbs);
  if (rc != 0) {
    *err = "nghttp2_session_client_new failed";
    return nullptr;
  }
  ch->session_ = session;
  nghttp2_settings_entry iv[3] = {
      {NGHTTP2_SETTINGS_ENABLE_PUSH, 0},
      {NGHTTP2_SETTINGS_INITIAL_WINDOW_SIZE, opts.initial_window},
      {NGHTTP2_SETTINGS_MAX_FRAME_SIZE, 1u << 20},
  };
  nghttp2_submit_settings(session, NGHTTP2_FLAG_NONE, iv, 3);
  nghttp2_session_set_local_window_size(session, NGHTTP2_FLAG_NONE, 0, static_cast<int32_t>(opts.initial_window));
  ch->evfd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  ch->last_activity_ns_ = NowNs();
  ch->io_ = std::thread([raw = ch.get()] { raw->Loop(); });
  return ch;
}

H2Channel::~H2Channel()
{
  stop_ = true;
  Wake();
  if (io_.joinable()) io_.join();
  if (session_) nghttp2_session_del(S(session_));
  if (evfd_ >= 0) close(evfd_);
}

void
H2Channel::Wake()
{
  uint64_t one = 1;
  ssize_t w = write(evfd_, &one, sizeof(one));
  (void)w;
}

void
H2Channel::Post(std::function<void()> fn)
{
  {
    std::lock_guard<std::mutex> lk(mu_);
    tasks_.push_back(std::move(fn));
  }
  Wake();
}

std::shared_ptr<H2Call>
H2Channel::StartCall(
    const std::string& path, const std::vector<std::pair<std::string, std::string>>& metadata, uint64_t timeout_us,
    GrpcCompression compression, H2CallHandlers handlers)
{
  auto call = std::make_shared<H2Call>();
  call->chan_ = shared_from_this();
  call->handlers_ = std::move(handlers);
  call->compression_ = compression;
  if (timeout_us) call->deadline_ns_ = NowNs() + timeout_us * 1000;
  if (dead_) {
    GrpcStatus st{14, "channel is broken: " + dead_reason_};
    if (call->handlers_.on_close) call->handlers_.on_close(st);
    return call;
  }
  std::vector<std::pair<std::string, std::string>> hdrs = {
      {":method", "POST"},
      {":scheme", opts_.tls.enabled ? "https" : "http"},
      {":path", path},
      {":authority", authority_},
      {"content-type", "application/grpc"},
      {"te", "trailers"},
      {"user-agent", "triton-mi355x-grpc/1.0"},
      {"grpc-accept-encoding", "identity,deflate,gzip"},
  };
  if (compression == GrpcCompression::GZIP) hdrs.push_back({"grpc-encoding", "gzip"});
  if (compression == GrpcCompression::DEFLATE) hdrs.push_back({"grpc-encoding", "deflate"});
  if (timeout_us) {
    if (timeout_us <= 99999999ull) hdrs.push_back({"grpc-timeout", std::to_string(timeout_us) + "u"});
    else hdrs.push_back({"grpc-timeout", std::to_string(std::min<uint64_t>(timeout_us / 1000, 99999999ull)) + "m"});
  }
  for (const auto& kv : metadata) {
    std::string k = kv.first;
    for (auto& c : k) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
    hdrs.push_back({k, kv.second});
  }
  Post([this, call, hdrs = std::move(hdrs)]() {
    if (call->cancelled_) {
      GrpcStatus st{1, "Locally cancelled by application!"};
      call->closed_ = true;
      if (call->handlers_.on_close) call->handlers_.on_close(st);
      return;
    }
    std::vector<nghttp2_nv> nva;
    nva.reserve(hdrs.size());
    for (const auto& h : hdrs) {
      nva.push_back({reinterpret_cast<uint8_t*>(const_cast<char*>(h.first.data())),
                     reinterpret_cast<uint8_t*>(const_cast<char*>(h.second.data())), h.first.size(), h.second.size(),
                     NGHTTP2_NV_FLAG_NONE});
    }
    nghttp2_data_provider prd;
    prd.source.ptr = this;
    prd.read_callback = cb_read_body;
    int32_t sid = nghttp2_submit_request(S(session_), nullptr, nva.data(), nva.size(), &prd, nullptr);
    if (sid < 0) {
      GrpcStatus st{14, std::string("failed to submit HTTP/2 request: ") + nghttp2_strerror(sid)};
      call->closed_ = true;
      if (call->handlers_.on_close) call->handlers_.on_close(st);
      return;
    }
    call->stream_id_ = sid;
    calls_[sid] = call;
  });
  return call;
}

void
H2Call::WriteFramed(std::string&& framed)
{
  auto ch = chan_.lock();
  if (!ch) return;
  auto self = shared_from_this();
  ch->Post([ch, self, framed = std::move(framed)]() mutable {
    self->out_.push_back(std::move(framed));
    if (self->deferred_ && self->stream_id_ > 0 && !self->closed_) {
      self->deferred_ = false;
      nghttp2_session_resume_data(S(ch->session_), self->stream_id_);
    }
  });
}

void
H2Call::Write(std::string&& message)
{
  auto ch = chan_.lock();
  if (!ch) return;
  std::string framed;
  GrpcFrame(message, compression_, &framed);
  auto self = shared_from_this();
  ch->Post([ch, self, framed = std::move(framed)]() mutable {
    self->out_.push_back(std::move(framed));
    if (self->deferred_ && self->stream_id_ > 0 && !self->closed_) {
      self->deferred_ = false;
      nghttp2_session_resume_data(S(ch->session_), self->stream_id_);
    }
  });
}

void
H2Call::WritesDone()
{
  auto ch = chan_.lock();
  if (!ch) return;
  auto self = shared_from_this();
  ch->Post([ch, self]() {
    self->writes_done_ = true;
    if (self->deferred_ && self->stream_id_ > 0 && !self->closed_) {
      self->deferred_ = false;
      nghttp2_session_resume_data(S(ch->session_), self->stream_id_);
    }
  });
}

void
H2Call::Cancel()
{
  auto ch = chan_.lock();
  if (!ch) return;
  auto self = shared_from_this();
  ch->Post([ch, self]() {
    if (self->closed_) return;
    self->cancelled_ = true;
    if (self->stream_id_ > 0) {
      nghttp2_submit_rst_stream(S(ch->session_), NGHTTP2_FLAG_NONE, self->stream_id_, NGHTTP2_CANCEL);
    }
  });
}

long
H2Channel::ReadBody(int32_t stream_id, uint8_t* buf, size_t length, uint32_t* data_flags)
{
  auto it = calls_.find(stream_id);
  if (it == calls_.end()) {
    *data_flags |= NGHTTP2_DATA_FLAG_EOF;
    return 0;
  }
  H2Call* c = it->second.get();
  size_t n = 0;
  while (n < length && !c->out_.empty()) {
    std::string& f = c->out_.front();
    size_t take = std::min(length - n, f.size() - c->out_pos_);
    std::memcpy(buf + n, f.data() + c->out_pos_, take);
    n += take;
    c->out_pos_ += take;
    if (c->out_pos_ == f.size()) {
      c->out_.pop_front();
      c->out_pos_ = 0;
    }
  }
  if (c->out_.empty() && c->writes_done_) {
    *data_flags |= NGHTTP2_DATA_FLAG_EOF;
    return static_cast<long>(n);
  }
  if (n == 0) {
    c->deferred_ = true;
    return NGHTTP2_ERR_DEFERRED;
  }
  return static_cast<long>(n);
}

void
H2Channel::OnHeader(int32_t stream_id, const std::string& name, const std::string& value)
{
  auto it = calls_.find(stream_id);
  if (it == calls_.end()) return;
  H2Call* c = it->second.get();
  if (name == ":status") {
    c->http_status_ = std::atoi(value.c_str());
  } else if (name == "grpc-status") {
    c->have_grpc_status_ = true;
    c->status_.code = std::atoi(value.c_str());
  } else if (name == "grpc-message") {
    c->status_.message = PercentDecode(value);
  } else if (name == "grpc-encoding") {
    c->resp_compressed_gzip_ = value == "gzip";
    c->resp_compressed_deflate_ = value == "deflate";
  }
}

void
H2Channel::OnData(int32_t stream_id, const uint8_t* data, size_t len)
{
  auto it = calls_.find(stream_id);
  if (it == calls_.end()) return;
  auto c = it->second;
  c->inbuf_.append(reinterpret_cast<const char*>(data), len);
  size_t pos = 0;
  while (c->inbuf_.size() - pos >= 5) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(c->inbuf_.data() + pos);
    uint32_t n = (static_cast<uint32_t>(p[1]) << 24) | (p[2] << 16) | (p[3] << 8) | p[4];
    if (c->inbuf_.size() - pos - 5 < n) break;
    std::string msg;
    if (p[0] & 1) {
      if (!Inflate(c->inbuf_.data() + pos + 5, n, &msg)) {
        c->status_ = GrpcStatus{13, "failed to decompress gRPC message"};
        c->have_grpc_status_ = true;
      }
    } else {
      msg.assign(c->inbuf_.data() + pos + 5, n);
    }
    pos += 5 + n;
    if (c->handlers_.on_message) c->handlers_.on_message(std::move(msg));
  }
  if (pos) c->inbuf_.erase(0, pos);
}

void
H2Channel::OnFrameRecv(int32_t, bool, bool)
{
  last_activity_ns_ = NowNs();
}

void
H2Channel::OnStreamClose(int32_t stream_id, uint32_t error_code)
{
  auto it = calls_.find(stream_id);
  if (it == calls_.end()) return;
  auto c = it->second;
  calls_.erase(it);
  if (c->closed_) return;
  c->closed_ = true;
  GrpcStatus st = c->status_;
  if (c->cancelled_ && (!c->have_grpc_status_ || st.code == 0)) {
    st = GrpcStatus{1, "Locally cancelled by application!"};
  } else if (!c->have_grpc_status_) {
    if (error_code != NGHTTP2_NO_ERROR) st = GrpcStatus{14, std::string("stream reset: ") + nghttp2_http2_strerror(error_code)};
    else if (c->http_status_ != 200) st = GrpcStatus{2, "HTTP status " + std::to_string(c->http_status_)};
    else st = GrpcStatus{13, "server closed the stream without a grpc-status"};
  }
  if (c->handlers_.on_close) c->handlers_.on_close(st);
}

void
H2Channel::FailAll(const std::string& why)
{
  dead_ = true;
  dead_reason_ = why;
  auto calls = std::move(calls_);
  calls_.clear();
  for (auto& kv : calls) {
    if (kv.second->closed_) continue;
    kv.second->closed_ = true;
    GrpcStatus st{14, why};
    if (kv.second->handlers_.on_close) kv.second->handlers_.on_close(st);
  }
}

bool
H2Channel::FlushSend()
{
  while (true) {
    if (sendpos_ >= sendbuf_.size()) {
      sendbuf_.clear();
      sendpos_ = 0;
      // gather everything nghttp2 wants to send (bounded per round)
      while (sendbuf_.size() < (4u << 20)) {
        const uint8_t* data;
        ssize_t n = nghttp2_session_mem_send(S(session_), &data);
        if (n < 0) return false;
        if (n == 0) break;
        sendbuf_.append(reinterpret_cast<const char*>(data), static_cast<size_t>(n));
      }
      if (sendbuf_.empty()) return true;
    }
    struct iovec v{const_cast<char*>(sendbuf_.data() + sendpos_), sendbuf_.size() - sendpos_};
    ssize_t w = sock_.Writev(&v, 1);
    if (w < 0) return false;
    if (w == 0) return true;  // would block; POLLOUT will resume
    sendpos_ += static_cast<size_t>(w);
  }
}

void
H2Channel::Loop()
{
  LoopBody();
  if (delete_on_exit_) {  // released by its last owner on this thread (see Create)
    io_.detach();
    delete this;
  }
}

void
H2Channel::LoopBody()
{
  char buf[1 << 17];
  while (!stop_) {
    std::deque<std::function<void()>> tasks;
    {
      std::lock_guard<std::mutex> lk(mu_);
      tasks.swap(tasks_);
    }
    for (auto& t : tasks) t();
    if (!dead_ && !FlushSend()) FailAll("connection write failed");
    // deadlines + keepalive
    uint64_t now = NowNs();
    int timeout_ms = 50;
    for (auto& kv : calls_) {
      auto& c = kv.second;
      if (c->deadline_ns_ && !c->closed_) {
        if (c->deadline_ns_ <= now) {
          c->closed_ = true;
          nghttp2_submit_rst_stream(S(session_), NGHTTP2_FLAG_NONE, c->stream_id_, NGHTTP2_CANCEL);
          GrpcStatus st{4, "Deadline Exceeded"};
          if (c->handlers_.on_close) c->handlers_.on_close(st);
        } else {
          timeout_ms = std::min<int>(timeout_ms, static_cast<int>((c->deadline_ns_ - now) / 1000000) + 1);
        }
      }
    }
    if (!dead_ && opts_.keepalive_time_ms < INT32_MAX) {
      bool idle_ok = opts_.keepalive_permit_without_calls || !calls_.empty();
      if (ping_sent_ns_ == 0 && idle_ok &&
          now - last_activity_ns_ > static_cast<uint64_t>(opts_.keepalive_time_ms) * 1000000ull) {
        nghttp2_submit_ping(S(session_), NGHTTP2_FLAG_NONE, nullptr);
        ping_sent_ns_ = now;
      } else if (ping_sent_ns_ && now - ping_sent_ns_ > static_cast<uint64_t>(opts_.keepalive_timeout_ms) * 1000000ull) {
        FailAll("keepalive ping timed out");
      }
    }
    if (!dead_ && !FlushSend()) FailAll("connection write failed");
    struct pollfd p[2];
    p[0].fd = sock_.fd();
    p[0].events = POLLIN | ((sendpos_ < sendbuf_.size()) ? POLLOUT : 0);
    p[0].revents = 0;
    p[1].fd = evfd_;
    p[1].events = POLLIN;
    p[1].revents = 0;
    int nfds = dead_ ? 1 : 2;
    struct pollfd* pp = dead_ ? &p[1] : p;
    int rc = ::poll(pp, nfds, timeout_ms);
    if (rc < 0) continue;
    if (p[1].revents & POLLIN) {
      uint64_t v;
      ssize_t r = read(evfd_, &v, sizeof(v));
      (void)r;
    }
    if (dead_) {
      // answer new calls immediately
      for (auto& kv : calls_) {
        if (!kv.second->closed_ && kv.second->handlers_.on_close) {
          kv.second->closed_ = true;
          kv.second->handlers_.on_close(GrpcStatus{14, dead_reason_});
        }
      }
      calls_.clear();
      continue;
    }
    if (p[0].revents & (POLLIN | POLLERR | POLLHUP)) {
      while (true) {
        ssize_t n = sock_.Read(buf, sizeof(buf));
        if (n == -2) break;
        if (n <= 0) {
          FailAll(n == 0 ? "connection closed by server" : "connection read failed");
          break;
        }
        last_activity_ns_ = NowNs();
        ssize_t used = nghttp2_session_mem_recv(S(session_), reinterpret_cast<const uint8_t*>(buf), static_cast<size_t>(n));
        if (used < 0) {
          FailAll(std::string("HTTP/2 protocol error: ") + nghttp2_strerror(static_cast<int>(used)));
          break;
        }
        if (static_cast<size_t>(n) < sizeof(buf) && !sock_.IsTls()) break;
      }
    }
    if (!dead_ && !FlushSend()) FailAll("connection write failed");
  }
}

}}  // namespace triton::client

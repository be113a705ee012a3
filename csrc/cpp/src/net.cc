// Socket / TLS / HTTP-1.1 response parsing / zlib / base64 (see net.h).
#include "net.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/ssl.h>
#include <poll.h>
#include <pthread.h>
#include <signal.h>
#include <sys/socket.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <chrono>
#include <cstring>

namespace triton { namespace client {

namespace {
// Blocks SIGPIPE on this thread for the guard's lifetime and discards one
// that a failed write raised meanwhile, leaving the process's handlers alone
// (a client library must not change global signal dispositions).
class SigpipeGuard {
 public:
  SigpipeGuard()
  {
    sigset_t pipe;
    sigemptyset(&pipe);
    sigaddset(&pipe, SIGPIPE);
    sigpending(&pending_before_);
    blocked_ = pthread_sigmask(SIG_BLOCK, &pipe, &old_) == 0;
  }
  ~SigpipeGuard()
  {
    if (!blocked_) return;
    if (!sigismember(&pending_before_, SIGPIPE)) {
      sigset_t pend;
      sigpending(&pend);
      if (sigismember(&pend, SIGPIPE)) {
        sigset_t pipe;
        sigemptyset(&pipe);
        sigaddset(&pipe, SIGPIPE);
        struct timespec zero = {0, 0};
        while (sigtimedwait(&pipe, nullptr, &zero) < 0 && errno == EINTR) {
        }
      }
    }
    pthread_sigmask(SIG_SETMASK, &old_, nullptr);
  }

 private:
  sigset_t old_, pending_before_;
  bool blocked_ = false;
};
}  // namespace


namespace {

uint64_t
NowNs()
{
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

std::string
Lower(std::string s)
{
  for (auto& c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return s;
}

}  // namespace

Socket::~Socket() { Close(); }

void
Socket::Close()
{
  if (ssl_) {
    SSL_shutdown(ssl_);
    SSL_free(ssl_);
    ssl_ = nullptr;
  }
  if (ctx_) {
    SSL_CTX_free(ctx_);
    ctx_ = nullptr;
  }
  if (fd_ >= 0) {
    ::close(fd_);
    fd_ = -1;
  }
}

void
Socket::SetNonBlocking(bool nb)
{
  int fl = fcntl(fd_, F_GETFL, 0);
  fcntl(fd_, F_SETFL, nb ? (fl | O_NONBLOCK) : (fl & ~O_NONBLOCK));
}

bool
Socket::Wait(bool for_write, int64_t timeout_us)
{
  if (ssl_ && !for_write && SSL_pending(ssl_) > 0) return true;
  struct pollfd p;
  p.fd = fd_;
  p.events = for_write ? POLLOUT : POLLIN;
  p.revents = 0;
  int ms = timeout_us <= 0 ? -1 : static_cast<int>((timeout_us + 999) / 1000);
  int rc;
  do {
    rc = ::poll(&p, 1, ms);
  } while (rc < 0 && errno == EINTR);
  return rc > 0;
}

std::string
Socket::Connect(const std::string& host, int port, uint64_t timeout_us, const TlsConfig& tls)
{
  Close();
  struct addrinfo hints;
  std::memset(&hints, 0, sizeof(hints));
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  struct addrinfo* res = nullptr;
  std::string port_s = std::to_string(port);
  int gai = getaddrinfo(host.c_str(), port_s.c_str(), &hints, &res);
  if (gai != 0) return std::string("failed to resolve ") + host + ": " + gai_strerror(gai);
  std::string err = "failed to connect to " + host + ":" + port_s;
  for (auto* ai = res; ai; ai = ai->ai_next) {
    int fd = ::socket(ai->ai_family, ai->ai_socktype | SOCK_CLOEXEC, ai->ai_protocol);
    if (fd < 0) continue;
    int fl = fcntl(fd, F_GETFL, 0);
    fcntl(fd, F_SETFL, fl | O_NONBLOCK);
    int rc = ::connect(fd, ai->ai_addr, ai->ai_addrlen);
    if (rc < 0 && errno == EINPROGRESS) {
      struct pollfd p{fd, POLLOUT, 0};
      int ms = timeout_us ? static_cast<int>((timeout_us + 999) / 1000) : -1;
      rc = ::poll(&p, 1, ms);
      int so_err = 0;
      socklen_t len = sizeof(so_err);
      if (rc > 0 && getsockopt(fd, SOL_SOCKET, SO_ERROR, &so_err, &len) == 0 && so_err == 0) {
        rc = 0;
      } else {
        rc = -1;
        if (so_err) err += std::string(": ") + std::strerror(so_err);
        else if (rc == 0) err += ": timeout";
      }
    }
    if (rc == 0) {
      fcntl(fd, F_SETFL, fl);  // back to blocking
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      int buf = 16 * 1024 * 1024;  // 16 MiB like the reference's curl buffers
      setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
      setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
      fd_ = fd;
      break;
    }
    ::close(fd);
  }
  freeaddrinfo(res);
  if (fd_ < 0) return err;
  if (tls.enabled) {
    ctx_ = SSL_CTX_new(TLS_client_method());
    if (!ctx_) return "SSL_CTX_new failed";
    if (!tls.ca_info.empty()) SSL_CTX_load_verify_locations(ctx_, tls.ca_info.c_str(), nullptr);
    else SSL_CTX_set_default_verify_paths(ctx_);
    if (!tls.cert.empty() &&
        SSL_CTX_use_certificate_file(ctx_, tls.cert.c_str(), tls.cert_der ? SSL_FILETYPE_ASN1 : SSL_FILETYPE_PEM) != 1)
      return "failed to load client certificate " + tls.cert;
    if (!tls.key.empty() &&
        SSL_CTX_use_PrivateKey_file(ctx_, tls.key.c_str(), tls.key_der ? SSL_FILETYPE_ASN1 : SSL_FILETYPE_PEM) != 1)
      return "failed to load client key " + tls.key;
    SSL_CTX_set_verify(ctx_, tls.verify_peer ? SSL_VERIFY_PEER : SSL_VERIFY_NONE, nullptr);
    if (!tls.alpn.empty() && tls.alpn.size() < 256) {
      std::string wire(1, static_cast<char>(tls.alpn.size()));
      wire += tls.alpn;
      SSL_CTX_set_alpn_protos(ctx_, reinterpret_cast<const unsigned char*>(wire.data()),
                              static_cast<unsigned>(wire.size()));
    }
    ssl_ = SSL_new(ctx_);
    SSL_set_fd(ssl_, fd_);
    SSL_set_tlsext_host_name(ssl_, host.c_str());
    if (tls.verify_host) SSL_set1_host(ssl_, host.c_str());
    int rc;
    {
      SigpipeGuard g;  // a peer that hangs up mid-handshake must not kill the process
      rc = SSL_connect(ssl_);
    }
    if (rc != 1) {
      char buf[256];
      ERR_error_string_n(ERR_get_error(), buf, sizeof(buf));
      Close();
      return std::string("TLS handshake failed: ") + buf;
    }
    if (!tls.alpn.empty()) {
      const unsigned char* got = nullptr;
      unsigned len = 0;
      SSL_get0_alpn_selected(ssl_, &got, &len);
      if (len != tls.alpn.size() || memcmp(got, tls.alpn.data(), len) != 0) {
        Close();
        return "TLS: server did not negotiate ALPN " + tls.alpn;
      }
    }
  }
  return "";
}

ssize_t
Socket::Writev(struct iovec* iov, int iovcnt)
{
  if (ssl_) {
    SigpipeGuard g;  // OpenSSL writes with write(2): a closed peer raises SIGPIPE
    ssize_t total = 0;
    for (int i = 0; i < iovcnt; ++i) {
      if (iov[i].iov_len == 0) continue;
      int n = SSL_write(ssl_, iov[i].iov_base, static_cast<int>(iov[i].iov_len));
      if (n <= 0) {
        int e = SSL_get_error(ssl_, n);
        if (e == SSL_ERROR_WANT_WRITE || e == SSL_ERROR_WANT_READ) return total;
        return -1;
      }
      total += n;
      if (static_cast<size_t>(n) < iov[i].iov_len) return total;
    }
    return total;
  }
  ssize_t n;
  struct msghdr mh;
  memset(&mh, 0, sizeof(mh));
  mh.msg_iov = iov;
  mh.msg_iovlen = std::min(iovcnt, 1024);
  do {
    n = ::sendmsg(fd_, &mh, MSG_NOSIGNAL);  // EPIPE instead of SIGPIPE on a closed peer
  } while (n < 0 && errno == EINTR);
  if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) return 0;
  return n;
}

ssize_t
Socket::Read(void* buf, size_t n)
{
  if (ssl_) {
    int r = SSL_read(ssl_, buf, static_cast<int>(n));
    if (r > 0) return r;
    int e = SSL_get_error(ssl_, r);
    if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) return -2;
    if (e == SSL_ERROR_ZERO_RETURN) return 0;
    return -1;
  }
  ssize_t r;
  do {
    r = ::read(fd_, buf, n);
  } while (r < 0 && errno == EINTR);
  if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) return -2;
  return r;
}

//==============================================================================
void
HttpResponseParser::Reset(bool head_request)
{
  state_ = State::Headers;
  head_.clear();
  headers_.clear();
  body_.clear();
  content_length_ = 0;
  has_length_ = false;
  status_ = 0;
  keep_alive_ = true;
  head_request_ = head_request;
  error_.clear();
  chunk_left_ = 0;
  chunk_phase_ = 0;
  line_.clear();
  first_byte_ns_ = 0;
}

bool
HttpResponseParser::ParseHeaders()
{
  size_t pos = head_.find("\r\n");
  std::string status_line = head_.substr(0, pos);
  if (status_line.compare(0, 5, "HTTP/") != 0) {
    error_ = "malformed HTTP status line";
    return false;
  }
  size_t sp = status_line.find(' ');
  status_ = std::strtol(status_line.c_str() + sp + 1, nullptr, 10);
  if (status_line.compare(0, 8, "HTTP/1.0") == 0) keep_alive_ = false;
  while (pos != std::string::npos && pos + 2 < head_.size()) {
    size_t next = head_.find("\r\n", pos + 2);
    std::string line = head_.substr(pos + 2, next == std::string::npos ? std::string::npos : next - pos - 2);
    size_t c = line.find(':');
    if (c != std::string::npos) {
      std::string k = Lower(line.substr(0, c));
      size_t vs = line.find_first_not_of(" \t", c + 1);
      std::string v = vs == std::string::npos ? "" : line.substr(vs);
      while (!v.empty() && (v.back() == ' ' || v.back() == '\t')) v.pop_back();
      headers_[k] = v;
    }
    pos = next;
  }
  auto it = headers_.find("connection");
  if (it != headers_.end()) {
    std::string v = Lower(it->second);
    if (v == "close") keep_alive_ = false;
    if (v == "keep-alive") keep_alive_ = true;
  }
  it = headers_.find("content-length");
  if (it != headers_.end()) {
    has_length_ = true;
    content_length_ = std::strtoull(it->second.c_str(), nullptr, 10);
  }
  return true;
}

size_t
HttpResponseParser::Feed(const char* data, size_t n)
{
  size_t used = 0;
  while (used < n && state_ != State::Done && state_ != State::Error) {
    if (state_ == State::Headers) {
      // scan for end of header block, keeping a 3-byte overlap
      size_t old = head_.size();
      head_.append(data + used, n - used);
      size_t from = old >= 3 ? old - 3 : 0;
      size_t e = head_.find("\r\n\r\n", from);
      if (e == std::string::npos) {
        used = n;
        if (head_.size() > (1u << 20)) {
          state_ = State::Error;
          error_ = "HTTP header block too large";
        }
        break;
      }
      size_t consumed_here = e + 4 - old;
      used += consumed_here;
      head_.resize(e + 2);
      if (!ParseHeaders()) {
        state_ = State::Error;
        break;
      }
      first_byte_ns_ = NowNs();
      bool no_body = head_request_ || status_ == 204 || status_ == 304 || (status_ >= 100 && status_ < 200);
      if (no_body) {
        state_ = State::Done;
      } else if (Lower(HeaderValue(headers_, "transfer-encoding")).find("chunked") != std::string::npos) {
        state_ = State::Chunked;
      } else if (has_length_) {
        body_.reserve(content_length_);
        state_ = content_length_ == 0 ? State::Done : State::Body;
      } else {
        keep_alive_ = false;
        state_ = State::Body;  // until close
        content_length_ = SIZE_MAX;
      }
    } else if (state_ == State::Body) {
      size_t want = std::min(n - used, content_length_ - body_.size());
      body_.append(data + used, want);
      used += want;
      if (body_.size() == content_length_) state_ = State::Done;
    } else if (state_ == State::Chunked) {
      if (chunk_phase_ == 1) {
        size_t want = std::min(n - used, chunk_left_);
        body_.append(data + used, want);
        used += want;
        chunk_left_ -= want;
        if (chunk_left_ == 0) chunk_phase_ = 2;
        continue;
      }
      char c = data[used++];
      line_.push_back(c);
      if (line_.size() >= 2 && line_[line_.size() - 2] == '\r' && c == '\n') {
        std::string l = line_.substr(0, line_.size() - 2);
        line_.clear();
        if (chunk_phase_ == 0) {
          chunk_left_ = std::strtoull(l.c_str(), nullptr, 16);
          chunk_phase_ = chunk_left_ ? 1 : 3;
        } else if (chunk_phase_ == 2) {
          chunk_phase_ = 0;
        } else if (chunk_phase_ == 3 && l.empty()) {
          state_ = State::Done;
        }
      }
    }
  }
  return used;
}

std::string
HeaderValue(const std::map<std::string, std::string>& h, const std::string& name)
{
  auto it = h.find(Lower(name));
  return it == h.end() ? std::string() : it->second;
}

//==============================================================================
bool
Compress(const std::vector<std::pair<const char*, size_t>>& parts, bool gzip, std::string* out)
{
  z_stream s;
  std::memset(&s, 0, sizeof(s));
  if (deflateInit2(&s, Z_DEFAULT_COMPRESSION, Z_DEFLATED, gzip ? (15 | 16) : 15, 8, Z_DEFAULT_STRATEGY) != Z_OK)
    return false;
  out->clear();
  char buf[1 << 16];
  for (size_t i = 0; i < parts.size(); ++i) {
    s.next_in = reinterpret_cast<Bytef*>(const_cast<char*>(parts[i].first));
    s.avail_in = static_cast<uInt>(parts[i].second);
    int flush = (i + 1 == parts.size()) ? Z_FINISH : Z_NO_FLUSH;
    do {
      s.next_out = reinterpret_cast<Bytef*>(buf);
      s.avail_out = sizeof(buf);
      int rc = deflate(&s, flush);
      if (rc == Z_STREAM_ERROR) {
        deflateEnd(&s);
        return false;
      }
      out->append(buf, sizeof(buf) - s.avail_out);
    } while (s.avail_out == 0);
  }
  if (parts.empty()) {
    s.next_out = reinterpret_cast<Bytef*>(buf);
    s.avail_out = sizeof(buf);
    deflate(&s, Z_FINISH);
    out->append(buf, sizeof(buf) - s.avail_out);
  }
  deflateEnd(&s);
  return true;
}

bool
Decompress(const std::string& in, std::string* out)
{
  z_stream s;
  std::memset(&s, 0, sizeof(s));
  // 15|32: auto-detect zlib or gzip header
  if (inflateInit2(&s, 15 | 32) != Z_OK) return false;
  s.next_in = reinterpret_cast<Bytef*>(const_cast<char*>(in.data()));
  s.avail_in = static_cast<uInt>(in.size());
  out->clear();
  char buf[1 << 16];
  int rc;
  do {
    s.next_out = reinterpret_cast<Bytef*>(buf);
    s.avail_out = sizeof(buf);
    rc = inflate(&s, Z_NO_FLUSH);
    if (rc != Z_OK && rc != Z_STREAM_END) {
      inflateEnd(&s);
      return false;
    }
    out->append(buf, sizeof(buf) - s.avail_out);
  } while (rc != Z_STREAM_END);
  inflateEnd(&s);
  return true;
}

static const char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

std::string
Base64Encode(const void* data, size_t n)
{
  const unsigned char* p = static_cast<const unsigned char*>(data);
  std::string out;
  out.reserve((n + 2) / 3 * 4);
  size_t i = 0;
  for (; i + 2 < n; i += 3) {
    uint32_t v = (p[i] << 16) | (p[i + 1] << 8) | p[i + 2];
    out.push_back(kB64[(v >> 18) & 63]);
    out.push_back(kB64[(v >> 12) & 63]);
    out.push_back(kB64[(v >> 6) & 63]);
    out.push_back(kB64[v & 63]);
  }
  if (i < n) {
    uint32_t v = p[i] << 16;
    if (i + 1 < n) v |= p[i + 1] << 8;
    out.push_back(kB64[(v >> 18) & 63]);
    out.push_back(kB64[(v >> 12) & 63]);
    out.push_back(i + 1 < n ? kB64[(v >> 6) & 63] : '=');
    out.push_back('=');
  }
  return out;
}

std::string
Base64EncodeLibb64(const void* data, size_t n)
{
  const std::string flat = Base64Encode(data, n);
  const size_t full = (n / 3) * 4;  // characters of complete 3-byte groups
  std::string out;
  out.reserve(flat.size() + full / 72 + 1);
  for (size_t i = 0; i < flat.size(); ++i) {
    out.push_back(flat[i]);
    if (i < full && (i + 1) % 72 == 0) out.push_back('\n');
  }
  out.push_back('\n');
  return out;
}

bool
Base64Decode(const std::string& in, std::string* out)
{
  int T[256];
  std::fill(T, T + 256, -1);
  for (int i = 0; i < 64; ++i) T[static_cast<unsigned char>(kB64[i])] = i;
  out->clear();
  uint32_t acc = 0;
  int bits = 0;
  for (unsigned char c : in) {
    if (c == '=' || c == '\n' || c == '\r' || c == ' ') continue;
    if (T[c] < 0) return false;
    acc = (acc << 6) | T[c];
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out->push_back(static_cast<char>((acc >> bits) & 0xff));
    }
  }
  return true;
}

std::string
UrlEncode(const std::string& s)
{
  std::string out;
  const char* hex = "0123456789ABCDEF";
  for (unsigned char c : s) {
    if (std::isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~') {
      out.push_back(static_cast<char>(c));
    } else {
      out.push_back('%');
      out.push_back(hex[c >> 4]);
      out.push_back(hex[c & 15]);
    }
  }
  return out;
}

}}  // namespace triton::client

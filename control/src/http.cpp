#include "http.hpp"

#ifdef _WIN32
#ifndef _WIN32_WINNT
#define _WIN32_WINNT 0x0601   // inet_pton, getaddrinfo
#endif
#include <winsock2.h>
#include <ws2tcpip.h>
#else
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <sys/socket.h>
#endif
#include <openssl/err.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <memory>
#include <sstream>

#include "platform.hpp"

namespace h2ok {

namespace {

std::string lower(std::string s) {
  for (auto& c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}

std::string ssl_err() {
  unsigned long e = ERR_get_error();
  if (!e) return "unknown TLS error";
  char buf[256];
  ERR_error_string_n(e, buf, sizeof buf);
  return buf;
}

bool is_ip_literal(const std::string& h) {
  unsigned char buf[16];
  return inet_pton(AF_INET, h.c_str(), buf) == 1 || inet_pton(AF_INET6, h.c_str(), buf) == 1;
}

class Conn {
 public:
  Conn(const Url& u, const TlsConfig& tls, double timeout_s) : timeout_s_(timeout_s) {
    connect_tcp(u.host, u.port);
    if (u.scheme == "https") start_tls(u.host, tls);
  }
  ~Conn() {
    if (ssl_) {
      SSL_shutdown(ssl_);
      SSL_free(ssl_);
    }
    if (ctx_) SSL_CTX_free(ctx_);
    plat::sock_close(fd_);
  }
  Conn(const Conn&) = delete;
  Conn& operator=(const Conn&) = delete;

  void write_all(const std::string& data) {
    size_t off = 0;
    while (off < data.size()) {
      long n;
      if (ssl_) {
        n = SSL_write(ssl_, data.data() + off, (int)(data.size() - off));
        if (n <= 0) throw HttpError("TLS write failed: " + ssl_err());
      } else {
        n = plat::sock_send(fd_, data.data() + off, data.size() - off);
        if (n < 0) throw HttpError("send failed: " + plat::sock_error());
      }
      off += (size_t)n;
    }
  }

  // read some bytes into buf_ (returns false on EOF / timeout)
  bool fill() {
    char tmp[16384];
    if (!(ssl_ && SSL_pending(ssl_) > 0)) {
      auto now = std::chrono::steady_clock::now();
      double left = timeout_s_ - std::chrono::duration<double>(now - start_).count();
      if (left <= 0) return false;
      int r = plat::sock_wait_readable(fd_, (int)(left * 1000) + 1);
      if (r <= 0) return false;
    }
    long n;
    if (ssl_) {
      n = SSL_read(ssl_, tmp, sizeof tmp);
      if (n <= 0) return false;
    } else {
      n = plat::sock_recv(fd_, tmp, sizeof tmp);
      if (n <= 0) return false;
    }
    buf_.append(tmp, (size_t)n);
    return true;
  }

  bool read_line(std::string& line) {
    while (true) {
      size_t p = buf_.find("\r\n");
      if (p != std::string::npos) {
        line = buf_.substr(0, p);
        buf_.erase(0, p + 2);
        return true;
      }
      if (!fill()) return false;
    }
  }

  bool read_exact(size_t n, std::string& out) {
    while (buf_.size() < n)
      if (!fill()) return false;
    out.append(buf_, 0, n);
    buf_.erase(0, n);
    return true;
  }

  std::string read_to_eof() {
    while (fill()) {
    }
    std::string out;
    out.swap(buf_);
    return out;
  }

  void reset_clock() { start_ = std::chrono::steady_clock::now(); }

 private:
  void connect_tcp(const std::string& host, int port) {
    plat::net_init();
    addrinfo hints{};
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    addrinfo* res = nullptr;
    int rc = getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res);
    if (rc != 0) throw HttpError("cannot resolve " + host + ": " + gai_strerror(rc));
    std::unique_ptr<addrinfo, void (*)(addrinfo*)> guard(res, freeaddrinfo);
    std::string last = "no address";
    for (addrinfo* a = res; a; a = a->ai_next) {
      plat::socket_t fd = plat::sock_open(a->ai_family, a->ai_socktype, a->ai_protocol);
      if (fd == plat::kBadSocket) continue;
      plat::sock_setup(fd, timeout_s_);
      if (plat::sock_connect(fd, a->ai_addr, a->ai_addrlen)) {
        fd_ = fd;
        return;
      }
      last = plat::sock_error();
      plat::sock_close(fd);
    }
    throw HttpError("cannot connect to " + host + ":" + std::to_string(port) + ": " + last);
  }

  void start_tls(const std::string& host, const TlsConfig& tls) {
    ctx_ = SSL_CTX_new(TLS_client_method());
    if (!ctx_) throw HttpError("SSL_CTX_new: " + ssl_err());
    SSL_CTX_set_min_proto_version(ctx_, TLS1_2_VERSION);
    if (!tls.ca_pem.empty()) {
      X509_STORE* store = SSL_CTX_get_cert_store(ctx_);
      BIO* bio = BIO_new_mem_buf(tls.ca_pem.data(), (int)tls.ca_pem.size());
      int added = 0;
      while (X509* x = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr)) {
        X509_STORE_add_cert(store, x);
        X509_free(x);
        ++added;
      }
      BIO_free(bio);
      ERR_clear_error();
      if (!added) throw HttpError("no certificate in certificate-authority data");
    } else {
      SSL_CTX_set_default_verify_paths(ctx_);
    }
    if (!tls.client_cert_pem.empty()) {
      BIO* bio = BIO_new_mem_buf(tls.client_cert_pem.data(), (int)tls.client_cert_pem.size());
      X509* x = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr);
      BIO_free(bio);
      if (!x || SSL_CTX_use_certificate(ctx_, x) != 1) throw HttpError("bad client certificate: " + ssl_err());
      X509_free(x);
      BIO* kb = BIO_new_mem_buf(tls.client_key_pem.data(), (int)tls.client_key_pem.size());
      EVP_PKEY* k = PEM_read_bio_PrivateKey(kb, nullptr, nullptr, nullptr);
      BIO_free(kb);
      if (!k || SSL_CTX_use_PrivateKey(ctx_, k) != 1) throw HttpError("bad client key: " + ssl_err());
      EVP_PKEY_free(k);
    }
    SSL_CTX_set_verify(ctx_, tls.insecure ? SSL_VERIFY_NONE : SSL_VERIFY_PEER, nullptr);
    ssl_ = SSL_new(ctx_);
    SSL_set_fd(ssl_, (int)fd_);
    const std::string name = tls.server_name.empty() ? host : tls.server_name;
    if (!is_ip_literal(name)) SSL_set_tlsext_host_name(ssl_, name.c_str());
    if (!tls.insecure) {
      X509_VERIFY_PARAM* vp = SSL_get0_param(ssl_);
      if (is_ip_literal(name)) X509_VERIFY_PARAM_set1_ip_asc(vp, name.c_str());
      else X509_VERIFY_PARAM_set1_host(vp, name.c_str(), 0);
    }
    if (SSL_connect(ssl_) != 1) throw HttpError("TLS handshake with " + host + " failed: " + ssl_err());
  }

  plat::socket_t fd_ = plat::kBadSocket;
  SSL_CTX* ctx_ = nullptr;
  SSL* ssl_ = nullptr;
  std::string buf_;
  double timeout_s_;
  std::chrono::steady_clock::time_point start_ = std::chrono::steady_clock::now();
};

std::string build_request(const Url& u, const HttpRequest& r, bool keep_open) {
  std::ostringstream os;
  std::string target = r.target.empty() ? "/" : r.target;
  os << r.method << ' ' << target << " HTTP/1.1\r\n";
  os << "Host: " << u.host;
  if (!((u.scheme == "http" && u.port == 80) || (u.scheme == "https" && u.port == 443))) os << ':' << u.port;
  os << "\r\n";
  bool has_ct = false, has_accept = false;
  for (auto& h : r.headers) {
    os << h.first << ": " << h.second << "\r\n";
    if (lower(h.first) == "content-type") has_ct = true;
    if (lower(h.first) == "accept") has_accept = true;
  }
  if (!has_accept) os << "Accept: application/json\r\n";
  os << "User-Agent: h2ok/0.1.0\r\n";
  if (!r.body.empty() || r.method == "POST" || r.method == "PUT" || r.method == "PATCH") {
    if (!has_ct) os << "Content-Type: application/json\r\n";
    os << "Content-Length: " << r.body.size() << "\r\n";
  }
  os << "Connection: " << (keep_open ? "keep-alive" : "close") << "\r\n\r\n";
  os << r.body;
  return os.str();
}

void read_head(Conn& c, HttpResponse& resp) {
  std::string line;
  if (!c.read_line(line)) throw HttpError("connection closed before response");
  // HTTP/1.1 200 OK
  size_t sp = line.find(' ');
  if (sp == std::string::npos) throw HttpError("bad status line: " + line);
  resp.status = std::atoi(line.c_str() + sp + 1);
  while (c.read_line(line)) {
    if (line.empty()) return;
    size_t colon = line.find(':');
    if (colon == std::string::npos) continue;
    std::string v = line.substr(colon + 1);
    size_t b = v.find_first_not_of(' ');
    resp.headers.emplace_back(line.substr(0, colon), b == std::string::npos ? "" : v.substr(b));
  }
  throw HttpError("connection closed inside headers");
}

}  // namespace

std::string HttpResponse::header(const std::string& name) const {
  std::string n = lower(name);
  for (auto& h : headers)
    if (lower(h.first) == n) return h.second;
  return "";
}

Url parse_url(const std::string& url) {
  Url u;
  size_t p = url.find("://");
  if (p == std::string::npos) throw HttpError("bad url: " + url);
  u.scheme = lower(url.substr(0, p));
  std::string rest = url.substr(p + 3);
  size_t slash = rest.find('/');
  std::string hostport = rest.substr(0, slash);
  u.path = slash == std::string::npos ? "" : rest.substr(slash);
  while (!u.path.empty() && u.path.back() == '/') u.path.pop_back();
  if (!hostport.empty() && hostport[0] == '[') {
    size_t rb = hostport.find(']');
    u.host = hostport.substr(1, rb - 1);
    if (rb + 1 < hostport.size() && hostport[rb + 1] == ':') u.port = std::atoi(hostport.c_str() + rb + 2);
  } else {
    size_t colon = hostport.rfind(':');
    if (colon != std::string::npos) {
      u.host = hostport.substr(0, colon);
      u.port = std::atoi(hostport.c_str() + colon + 1);
    } else {
      u.host = hostport;
    }
  }
  if (u.port == 0) u.port = u.scheme == "https" ? 443 : 80;
  return u;
}

HttpResponse http_request(const Url& server, const HttpRequest& req, const TlsConfig& tls) {
  Conn c(server, tls, req.timeout_s);
  c.write_all(build_request(server, req, false));
  HttpResponse resp;
  read_head(c, resp);
  std::string te = lower(resp.header("Transfer-Encoding"));
  std::string cl = resp.header("Content-Length");
  if (req.method == "HEAD" || resp.status == 204 || resp.status == 304) return resp;
  if (te.find("chunked") != std::string::npos) {
    std::string line;
    while (c.read_line(line)) {
      size_t sz = std::strtoul(line.c_str(), nullptr, 16);
      if (sz == 0) {
        c.read_line(line);
        break;
      }
      if (!c.read_exact(sz, resp.body)) throw HttpError("truncated chunk");
      c.read_line(line);
    }
  } else if (!cl.empty()) {
    if (!c.read_exact(std::strtoul(cl.c_str(), nullptr, 10), resp.body)) throw HttpError("truncated body");
  } else {
    resp.body = c.read_to_eof();
  }
  return resp;
}

int http_stream_lines(const Url& server, const HttpRequest& req, const TlsConfig& tls,
                      const std::function<bool(const std::string&)>& on_line) {
  Conn c(server, tls, req.timeout_s);
  c.write_all(build_request(server, req, false));
  HttpResponse resp;
  read_head(c, resp);
  bool chunked = lower(resp.header("Transfer-Encoding")).find("chunked") != std::string::npos;
  std::string pending;
  auto emit = [&](const std::string& data) -> bool {
    pending += data;
    size_t p;
    while ((p = pending.find('\n')) != std::string::npos) {
      std::string ln = pending.substr(0, p);
      pending.erase(0, p + 1);
      if (!ln.empty() && ln.back() == '\r') ln.pop_back();
      if (!ln.empty() && !on_line(ln)) return false;
    }
    return true;
  };
  if (chunked) {
    std::string line;
    while (c.read_line(line)) {
      size_t sz = std::strtoul(line.c_str(), nullptr, 16);
      if (sz == 0) break;
      std::string data;
      if (!c.read_exact(sz, data)) break;
      c.read_line(line);
      if (!emit(data)) return resp.status;
    }
  } else {
    std::string cl = resp.header("Content-Length");
    std::string body = cl.empty() ? c.read_to_eof() : std::string();
    if (!cl.empty()) c.read_exact(std::strtoul(cl.c_str(), nullptr, 10), body);
    if (!emit(body)) return resp.status;
  }
  if (!pending.empty()) on_line(pending);
  return resp.status;
}

std::string url_encode(const std::string& s) {
  static const char* hex = "0123456789ABCDEF";
  std::string out;
  for (unsigned char c : s) {
    if (std::isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~') {
      out += (char)c;
    } else {
      out += '%';
      out += hex[c >> 4];
      out += hex[c & 15];
    }
  }
  return out;
}

std::string base64_encode(const std::string& in) {
  static const char* tbl = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string out;
  size_t i = 0;
  while (i + 2 < in.size()) {
    uint32_t v = ((uint8_t)in[i] << 16) | ((uint8_t)in[i + 1] << 8) | (uint8_t)in[i + 2];
    out += tbl[v >> 18];
    out += tbl[(v >> 12) & 63];
    out += tbl[(v >> 6) & 63];
    out += tbl[v & 63];
    i += 3;
  }
  if (i + 1 == in.size()) {
    uint32_t v = (uint8_t)in[i] << 16;
    out += tbl[v >> 18];
    out += tbl[(v >> 12) & 63];
    out += "==";
  } else if (i + 2 == in.size()) {
    uint32_t v = ((uint8_t)in[i] << 16) | ((uint8_t)in[i + 1] << 8);
    out += tbl[v >> 18];
    out += tbl[(v >> 12) & 63];
    out += tbl[(v >> 6) & 63];
    out += '=';
  }
  return out;
}

std::string base64_decode(const std::string& in) {
  auto val = [](char c) -> int {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+' || c == '-') return 62;
    if (c == '/' || c == '_') return 63;
    return -1;
  };
  std::string out;
  uint32_t acc = 0;
  int bits = 0;
  for (char c : in) {
    int v = val(c);
    if (v < 0) continue;
    acc = (acc << 6) | (uint32_t)v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out += (char)((acc >> bits) & 0xFF);
    }
  }
  return out;
}

}  // namespace h2ok

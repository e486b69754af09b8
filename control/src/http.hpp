// Small HTTP/1.1 client (plain TCP or TLS via OpenSSL) used to talk to the
// Kubernetes API server: JSON requests, chunked responses and long-poll
// watch streams (newline-delimited JSON events).  Replaces the reference's
// kube-rs/hyper/vendored-OpenSSL stack (Cargo.toml:9,21 of
// isgasho/h2o-kubernetes) with a dependency-free native implementation.
#pragma once

#include <functional>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace h2ok {

struct Url {
  std::string scheme;  // http | https
  std::string host;
  int port = 0;
  std::string path;  // includes leading '/' and base path of the server url
};

Url parse_url(const std::string& url);

struct TlsConfig {
  std::string ca_pem;           // trusted CA bundle (PEM); empty = system default
  bool insecure = false;        // skip server verification
  std::string client_cert_pem;  // mTLS client certificate
  std::string client_key_pem;
  std::string server_name;      // override SNI / verification name
};

struct HttpResponse {
  int status = 0;
  std::vector<std::pair<std::string, std::string>> headers;
  std::string body;
  std::string header(const std::string& name) const;
};

class HttpError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

struct HttpRequest {
  std::string method = "GET";
  std::string target;  // path + query
  std::vector<std::pair<std::string, std::string>> headers;
  std::string body;
  double timeout_s = 30.0;
};

// One request on a fresh connection.
HttpResponse http_request(const Url& server, const HttpRequest& req, const TlsConfig& tls);

// Streaming request: calls on_line for each newline-delimited chunk of the
// body until it returns false, the server closes, or timeout_s elapses.
// Returns the HTTP status.
int http_stream_lines(const Url& server, const HttpRequest& req, const TlsConfig& tls,
                      const std::function<bool(const std::string&)>& on_line);

std::string url_encode(const std::string& s);
std::string base64_encode(const std::string& in);
std::string base64_decode(const std::string& in);

}  // namespace h2ok

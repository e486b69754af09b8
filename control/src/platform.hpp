// Operating-system layer of the control plane (h2ok CLI + operator): the few
// calls that differ between POSIX (Linux, macOS) and Windows.  The reference
// ships h2ok for all three (/root/reference/.github/workflows/release.yml:14,31,101);
// everything above this file is portable C++17 + OpenSSL.
#pragma once

#include <cstdint>
#include <ctime>
#include <string>
#include <utility>
#include <vector>

namespace h2ok::plat {

// stdout is an interactive terminal (h2ok prints the human messages then,
// the bare descriptor file name when piped)
bool stdout_is_tty();

bool is_regular_file(const std::string& path);
bool path_exists(const std::string& path);
std::string current_dir();
char path_sep();

// Run argv with extra environment; stdout / stderr captured; killed after
// timeout_s.  Returns the exit status (-1: could not run / timed out).
int run_capture(const std::vector<std::string>& argv, const std::vector<std::pair<std::string, std::string>>& env,
                std::string& out, std::string& err, double timeout_s);

// "YYYY-MM-DDTHH:MM:SS..." (RFC 3339, UTC) -> seconds since the epoch (0 = unparsable)
long long parse_rfc3339_utc(const std::string& t);

// ---- TCP sockets -----------------------------------------------------------
using socket_t = std::intptr_t;
constexpr socket_t kBadSocket = -1;

void net_init();  // idempotent (WSAStartup on Windows)
socket_t sock_open(int family, int type, int proto);
bool sock_connect(socket_t s, const void* addr, std::size_t len);
void sock_close(socket_t s);
void sock_setup(socket_t s, double timeout_s);   // send timeout, TCP_NODELAY, no SIGPIPE
long sock_send(socket_t s, const char* data, std::size_t n);   // < 0 on error (EINTR retried)
long sock_recv(socket_t s, char* data, std::size_t n);
int sock_wait_readable(socket_t s, int timeout_ms);   // > 0 readable, 0 timeout, < 0 error
std::string sock_error();

}  // namespace h2ok::plat

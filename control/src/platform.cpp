#include "platform.hpp"

#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>

#ifdef _WIN32
#ifndef _WIN32_WINNT
#define _WIN32_WINNT 0x0601   // WSAPoll, inet_pton
#endif
#include <winsock2.h>
#include <ws2tcpip.h>
#include <direct.h>
#include <io.h>
#include <windows.h>
#else
#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cerrno>
#endif

namespace h2ok::plat {

// ---- files / terminal -----------------------------------------------------------
bool stdout_is_tty() {
#ifdef _WIN32
  return _isatty(_fileno(stdout)) != 0;
#else
  return ::isatty(STDOUT_FILENO) == 1;
#endif
}

bool is_regular_file(const std::string& p) {
  struct stat st{};
  return ::stat(p.c_str(), &st) == 0 && (st.st_mode & S_IFMT) == S_IFREG;
}

bool path_exists(const std::string& p) {
  struct stat st{};
  return ::stat(p.c_str(), &st) == 0;
}

std::string current_dir() {
  char buf[4096];
#ifdef _WIN32
  return _getcwd(buf, sizeof buf) ? std::string(buf) : std::string(".");
#else
  return ::getcwd(buf, sizeof buf) ? std::string(buf) : std::string(".");
#endif
}

char path_sep() {
#ifdef _WIN32
  return '\\';
#else
  return '/';
#endif
}

long long parse_rfc3339_utc(const std::string& t) {
  int Y = 0, M = 0, D = 0, h = 0, m = 0, s = 0;
  if (t.size() < 19 || std::sscanf(t.c_str(), "%4d-%2d-%2dT%2d:%2d:%2d", &Y, &M, &D, &h, &m, &s) != 6) return 0;
  // days from civil (proleptic Gregorian), no timegm / _mkgmtime dependency
  const int y = Y - (M <= 2);
  const int era = (y >= 0 ? y : y - 399) / 400;
  const unsigned yoe = (unsigned)(y - era * 400);
  const unsigned doy = (153u * (unsigned)(M + (M > 2 ? -3 : 9)) + 2u) / 5u + (unsigned)D - 1u;
  const unsigned doe = yoe * 365u + yoe / 4u - yoe / 100u + doy;
  const long long days = (long long)era * 146097LL + (long long)doe - 719468LL;
  return days * 86400LL + h * 3600LL + m * 60LL + s;
}

// ---- child processes ------------------------------------------------------------
#ifdef _WIN32
static std::string quote_arg(const std::string& a) {
  if (!a.empty() && a.find_first_of(" \t\"") == std::string::npos) return a;
  std::string q = "\"";
  int bs = 0;
  for (char c : a) {
    if (c == '\\') { ++bs; continue; }
    if (c == '"') q.append(2 * bs + 1, '\\');
    else q.append(bs, '\\');
    bs = 0;
    q.push_back(c);
  }
  q.append(2 * bs, '\\');
  q.push_back('"');
  return q;
}

int run_capture(const std::vector<std::string>& argv, const std::vector<std::pair<std::string, std::string>>& env,
                std::string& out, std::string& err, double timeout_s) {
  if (argv.empty()) return -1;
  SECURITY_ATTRIBUTES sa{sizeof(SECURITY_ATTRIBUTES), nullptr, TRUE};
  HANDLE or_ = nullptr, ow = nullptr, er = nullptr, ew = nullptr;
  if (!CreatePipe(&or_, &ow, &sa, 0)) return -1;
  if (!CreatePipe(&er, &ew, &sa, 0)) {
    CloseHandle(or_);
    CloseHandle(ow);
    return -1;
  }
  SetHandleInformation(or_, HANDLE_FLAG_INHERIT, 0);
  SetHandleInformation(er, HANDLE_FLAG_INHERIT, 0);
  // environment block: ours with the extras REPLACING inherited entries of the
  // same name (Windows names are case-insensitive and a block with duplicates
  // resolves to the first one), sorted case-insensitively as CreateProcess expects
  struct CiLess {
    bool operator()(const std::string& a, const std::string& b) const {
      return _stricmp(a.c_str(), b.c_str()) < 0;
    }
  };
  std::map<std::string, std::string, CiLess> vars;
  if (LPCH cur = GetEnvironmentStringsA()) {
    for (LPCH p = cur; *p; p += std::strlen(p) + 1) {
      const std::string e(p);
      const size_t eq = e.find('=', 1);   // "=C:=C:\dir" drive entries start with '='
      if (eq == std::string::npos) continue;
      vars.emplace(e.substr(0, eq), e.substr(eq + 1));
    }
    FreeEnvironmentStringsA(cur);
  }
  for (auto& [k, v] : env) vars[k] = v;
  std::string block;
  for (auto& [k, v] : vars) block.append(k + "=" + v).push_back('\0');
  block.push_back('\0');
  std::string cmd;
  for (auto& a : argv) cmd += (cmd.empty() ? "" : " ") + quote_arg(a);
  STARTUPINFOA si{};
  si.cb = sizeof si;
  si.dwFlags = STARTF_USESTDHANDLES;
  si.hStdOutput = ow;
  si.hStdError = ew;
  si.hStdInput = GetStdHandle(STD_INPUT_HANDLE);
  PROCESS_INFORMATION pi{};
  std::vector<char> cmdline(cmd.begin(), cmd.end());
  cmdline.push_back('\0');
  // the child and every helper it spawns live in one job object that is killed
  // as a whole on timeout (and when the handle closes): a helper that inherited
  // the pipe's write end can then never keep the reads below waiting
  HANDLE job = CreateJobObjectA(nullptr, nullptr);
  if (job) {
    JOBOBJECT_EXTENDED_LIMIT_INFORMATION li{};
    li.BasicLimitInformation.LimitFlags = JOB_OBJECT_LIMIT_KILL_ON_JOB_CLOSE;
    SetInformationJobObject(job, JobObjectExtendedLimitInformation, &li, sizeof li);
  }
  const BOOL ok = CreateProcessA(nullptr, cmdline.data(), nullptr, nullptr, TRUE, CREATE_NO_WINDOW | CREATE_SUSPENDED,
                                 block.data(), nullptr, &si, &pi);
  CloseHandle(ow);
  CloseHandle(ew);
  if (!ok) {
    if (job) CloseHandle(job);
    CloseHandle(or_);
    CloseHandle(er);
    return -1;
  }
  if (job) AssignProcessToJobObject(job, pi.hProcess);
  ResumeThread(pi.hThread);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds((long long)(timeout_s * 1000));
  bool timed_out = false;
  char buf[4096];
  HANDLE hs[2] = {or_, er};
  std::string* dst[2] = {&out, &err};
  while (true) {
    bool any = false;
    for (int i = 0; i < 2; ++i) {
      DWORD avail = 0;
      if (hs[i] && PeekNamedPipe(hs[i], nullptr, 0, nullptr, &avail, nullptr) && avail > 0) {
        DWORD n = 0;
        if (ReadFile(hs[i], buf, (DWORD)std::min<DWORD>(avail, sizeof buf), &n, nullptr) && n > 0) {
          dst[i]->append(buf, n);
          any = true;
        }
      }
    }
    if (WaitForSingleObject(pi.hProcess, 0) == WAIT_OBJECT_0 && !any) break;
    if (std::chrono::steady_clock::now() > deadline) {
      timed_out = true;
      if (job) TerminateJobObject(job, 1);
      else TerminateProcess(pi.hProcess, 1);
      break;
    }
    if (!any) Sleep(5);
  }
  // drain what is already buffered, never blocking: only what PeekNamedPipe
  // reports, for at most 200 ms (a surviving grandchild may hold the pipe open)
  const auto drain_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(200);
  for (bool more = true; more && std::chrono::steady_clock::now() < drain_end;) {
    more = false;
    for (int i = 0; i < 2; ++i) {
      DWORD avail = 0, n = 0;
      if (PeekNamedPipe(hs[i], nullptr, 0, nullptr, &avail, nullptr) && avail > 0 &&
          ReadFile(hs[i], buf, (DWORD)std::min<DWORD>(avail, sizeof buf), &n, nullptr) && n > 0) {
        dst[i]->append(buf, n);
        more = true;
      }
    }
  }
  DWORD code = 1;
  WaitForSingleObject(pi.hProcess, timed_out ? 5000 : INFINITE);
  GetExitCodeProcess(pi.hProcess, &code);
  CloseHandle(pi.hProcess);
  CloseHandle(pi.hThread);
  CloseHandle(or_);
  CloseHandle(er);
  if (job) CloseHandle(job);   // KILL_ON_JOB_CLOSE: no helper outlives the call
  return timed_out ? -1 : (int)code;
}
#else
int run_capture(const std::vector<std::string>& argv, const std::vector<std::pair<std::string, std::string>>& env,
                std::string& out, std::string& err, double timeout_s) {
  int po[2], pe[2];
  if (pipe(po) != 0) return -1;
  if (pipe(pe) != 0) {
    close(po[0]);
    close(po[1]);
    return -1;
  }
  pid_t pid = fork();
  if (pid < 0) return -1;
  if (pid == 0) {
    dup2(po[1], 1);
    dup2(pe[1], 2);
    close(po[0]);
    close(pe[0]);
    int devnull = open("/dev/null", O_RDONLY);
    if (devnull >= 0) dup2(devnull, 0);
    for (auto& [k, v] : env) setenv(k.c_str(), v.c_str(), 1);
    std::vector<char*> av;
    for (auto& a : argv) av.push_back(const_cast<char*>(a.c_str()));
    av.push_back(nullptr);
    execvp(av[0], av.data());
    std::fprintf(stderr, "exec %s: %s\n", av[0], std::strerror(errno));
    _exit(127);
  }
  close(po[1]);
  close(pe[1]);
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds((long long)(timeout_s * 1000));
  struct pollfd fds[2] = {{po[0], POLLIN, 0}, {pe[0], POLLIN, 0}};
  int open_fds = 2;
  bool timed_out = false;
  char buf[4096];
  while (open_fds > 0) {
    auto left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now());
    if (left.count() <= 0) {
      timed_out = true;
      break;
    }
    if (poll(fds, 2, (int)left.count()) <= 0) continue;
    for (int i = 0; i < 2; ++i) {
      if (fds[i].fd < 0 || !(fds[i].revents & (POLLIN | POLLHUP | POLLERR))) continue;
      ssize_t n = read(fds[i].fd, buf, sizeof buf);
      if (n > 0) {
        (i == 0 ? out : err).append(buf, (size_t)n);
      } else {
        close(fds[i].fd);
        fds[i].fd = -1;
        --open_fds;
      }
    }
  }
  for (auto& f : fds)
    if (f.fd >= 0) close(f.fd);
  if (timed_out) kill(pid, SIGKILL);
  int st = 0;
  waitpid(pid, &st, 0);
  if (timed_out) return -1;
  return WIFEXITED(st) ? WEXITSTATUS(st) : -1;
}
#endif

// ---- sockets ------------------------------------------------------------------------
void net_init() {
#ifdef _WIN32
  static bool done = [] {
    WSADATA w;
    return WSAStartup(MAKEWORD(2, 2), &w) == 0;
  }();
  (void)done;
#endif
}

socket_t sock_open(int family, int type, int proto) {
  net_init();
#ifdef _WIN32
  SOCKET s = ::socket(family, type, proto);
  return s == INVALID_SOCKET ? kBadSocket : (socket_t)s;
#else
  int s = ::socket(family, type, proto);
  return s < 0 ? kBadSocket : (socket_t)s;
#endif
}

bool sock_connect(socket_t s, const void* addr, std::size_t len) {
#ifdef _WIN32
  return ::connect((SOCKET)s, (const sockaddr*)addr, (int)len) == 0;
#else
  return ::connect((int)s, (const sockaddr*)addr, (socklen_t)len) == 0;
#endif
}

void sock_close(socket_t s) {
  if (s == kBadSocket) return;
#ifdef _WIN32
  ::closesocket((SOCKET)s);
#else
  ::close((int)s);
#endif
}

void sock_setup(socket_t s, double timeout_s) {
  int one = 1;
#ifdef _WIN32
  DWORD ms = (DWORD)(timeout_s * 1000);
  setsockopt((SOCKET)s, SOL_SOCKET, SO_SNDTIMEO, (const char*)&ms, sizeof ms);
  setsockopt((SOCKET)s, IPPROTO_TCP, TCP_NODELAY, (const char*)&one, sizeof one);
#else
  timeval tv{};
  tv.tv_sec = (long)timeout_s;
  tv.tv_usec = (long)((timeout_s - (long)timeout_s) * 1e6);
  setsockopt((int)s, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
  setsockopt((int)s, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
#ifdef SO_NOSIGPIPE
  // macOS has no MSG_NOSIGNAL: a closed peer must not SIGPIPE the CLI
  setsockopt((int)s, SOL_SOCKET, SO_NOSIGPIPE, &one, sizeof one);
#endif
#endif
}

long sock_send(socket_t s, const char* data, std::size_t n) {
#ifdef _WIN32
  return (long)::send((SOCKET)s, data, (int)n, 0);
#else
#ifndef MSG_NOSIGNAL
#define MSG_NOSIGNAL 0
#endif
  while (true) {
    ssize_t r = ::send((int)s, data, n, MSG_NOSIGNAL);
    if (r < 0 && errno == EINTR) continue;
    return (long)r;
  }
#endif
}

long sock_recv(socket_t s, char* data, std::size_t n) {
#ifdef _WIN32
  return (long)::recv((SOCKET)s, data, (int)n, 0);
#else
  return (long)::recv((int)s, data, n, 0);
#endif
}

int sock_wait_readable(socket_t s, int timeout_ms) {
#ifdef _WIN32
  WSAPOLLFD p{(SOCKET)s, POLLRDNORM, 0};
  return WSAPoll(&p, 1, timeout_ms);
#else
  pollfd p{(int)s, POLLIN, 0};
  return ::poll(&p, 1, timeout_ms);
#endif
}

std::string sock_error() {
#ifdef _WIN32
  return "winsock error " + std::to_string(WSAGetLastError());
#else
  return std::strerror(errno);
#endif
}

}  // namespace h2ok::plat

// Multi-threaded CSV / SVMLight-free delimited-text parser (host C++).
//
// Equivalent of H2O-3's ParseSetup + Parse (the reference deploys the Java
// image that provides them, templates.rs:30 of isgasho/h2o-kubernetes):
//   * separator / header / column type guessing on a sample (numeric, enum
//     (categorical), string), H2O-style NA tokens;
//   * a parallel parse of the whole file split at line boundaries into
//     per-thread chunks; numeric columns land in float64 arrays, categorical
//     columns in int32 codes against a lexicographically sorted domain (H2O
//     domain order);
//   * an optional byte range [start, end) so every rank of a distributed
//     cluster parses only its own shard of a shared file.
// Exposed as a flat C ABI for ctypes.
#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#define H2OMX_HOST_API extern "C" __attribute__((visibility("default")))

namespace {

enum ColType { kNumeric = 0, kEnum = 1, kString = 2 };

bool is_na_token(const char* b, size_t n) {
  if (n == 0) return true;
  static const char* toks[] = {"NA", "N/A", "na", "n/a", "NaN", "nan", "null", "NULL", "?", "-", ""};
  for (const char* t : toks)
    if (std::strlen(t) == n && std::memcmp(t, b, n) == 0) return true;
  return false;
}

bool parse_double(const char* b, size_t n, double& out) {
  if (n == 0) return false;
  char buf[64];
  if (n >= sizeof buf) return false;
  std::memcpy(buf, b, n);
  buf[n] = 0;
  char* end = nullptr;
  errno = 0;
  out = std::strtod(buf, &end);
  if (end == buf) return false;
  while (*end == ' ' || *end == '\t') ++end;
  return *end == 0;
}

struct Field {
  const char* b;
  size_t n;
};

// split one line into fields (RFC-4180 quotes; quotes are stripped, "" -> ")
void split_line(const char* b, const char* e, char sep, std::vector<Field>& out, std::vector<std::string>& scratch) {
  out.clear();
  scratch.clear();
  const char* p = b;
  while (true) {
    while (p < e && (*p == ' ') && sep != ' ') ++p;
    if (p < e && *p == '"') {
      std::string s;
      ++p;
      while (p < e) {
        if (*p == '"') {
          if (p + 1 < e && p[1] == '"') {
            s += '"';
            p += 2;
            continue;
          }
          ++p;
          break;
        }
        s += *p++;
      }
      while (p < e && *p != sep) ++p;
      scratch.push_back(std::move(s));
      out.push_back({nullptr, scratch.size() - 1});  // index into scratch
    } else {
      const char* st = p;
      while (p < e && *p != sep) ++p;
      const char* en = p;
      while (en > st && (en[-1] == ' ' || en[-1] == '\r' || en[-1] == '\t')) --en;
      out.push_back({st, (size_t)(en - st)});
    }
    if (p >= e) break;
    ++p;  // skip separator
    if (sep == ' ')
      while (p < e && *p == ' ') ++p;
  }
  // resolve quoted fields to stable pointers
  for (auto& f : out)
    if (!f.b) {
      const std::string& s = scratch[f.n];
      f.b = s.data();
      f.n = s.size();
    }
}

struct Parsed {
  std::vector<std::string> names;
  std::vector<int> types;
  std::vector<std::vector<double>> num;       // per numeric column
  std::vector<std::vector<int32_t>> codes;    // per enum/string column
  std::vector<std::vector<std::string>> domains;
  int64_t nrows = 0;
  char sep = ',';
  int header = 0;
  std::string error;
};

char guess_sep(const std::string& line) {
  const char cands[] = {',', '\t', ';', '|', ' '};
  char best = ',';
  size_t bestc = 0;
  for (char c : cands) {
    size_t k = std::count(line.begin(), line.end(), c);
    if (k > bestc) {
      bestc = k;
      best = c;
    }
  }
  return best;
}

std::vector<std::pair<const char*, const char*>> lines_of(const char* b, const char* e) {
  std::vector<std::pair<const char*, const char*>> out;
  const char* p = b;
  while (p < e) {
    const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(e - p)));
    const char* le = nl ? nl : e;
    const char* lb = p;
    const char* lt = le;
    if (lt > lb && lt[-1] == '\r') --lt;
    if (lt > lb) out.push_back({lb, lt});
    p = nl ? nl + 1 : e;
  }
  return out;
}

Parsed* parse_buffer(const std::string& data, char sep, int header, int nthreads, const std::vector<int>& forced) {
  auto* P = new Parsed();
  const char* b = data.data();
  const char* e = b + data.size();
  auto lines = lines_of(b, e);
  // drop comment lines
  lines.erase(std::remove_if(lines.begin(), lines.end(), [](auto& l) { return *l.first == '#'; }), lines.end());
  if (lines.empty()) {
    P->error = "empty file";
    return P;
  }
  std::string first(lines[0].first, lines[0].second);
  if (!sep) sep = guess_sep(first);
  P->sep = sep;
  std::vector<Field> f0, f1;
  std::vector<std::string> sc0, sc1;
  split_line(lines[0].first, lines[0].second, sep, f0, sc0);
  const size_t ncol = f0.size();
  if (header < 0) {
    // header if the first row is all non-numeric while some later row has numbers in those columns
    int first_nonnum = 0, later_num = 0;
    double d;
    for (auto& f : f0) first_nonnum += !parse_double(f.b, f.n, d) && !is_na_token(f.b, f.n);
    if (lines.size() > 1) {
      split_line(lines[1].first, lines[1].second, sep, f1, sc1);
      for (size_t j = 0; j < f1.size() && j < ncol; ++j) later_num += parse_double(f1[j].b, f1[j].n, d);
    }
    header = (first_nonnum == (int)ncol || (first_nonnum > 0 && later_num > 0)) ? 1 : 0;
  }
  P->header = header;
  for (size_t j = 0; j < ncol; ++j)
    P->names.push_back(header ? std::string(f0[j].b, f0[j].n) : "C" + std::to_string(j + 1));
  const size_t start = header ? 1 : 0;
  const size_t nl = lines.size() - start;
  P->nrows = (int64_t)nl;
  // type guess on a sample: numeric if every non-NA token parses
  std::vector<int> types(ncol, kNumeric);
  {
    std::vector<Field> fs;
    std::vector<std::string> scr;
    double d;
    size_t sample = std::min<size_t>(nl, 20000);
    for (size_t i = 0; i < sample; ++i) {
      split_line(lines[start + i].first, lines[start + i].second, sep, fs, scr);
      for (size_t j = 0; j < ncol && j < fs.size(); ++j)
        if (types[j] == kNumeric && !is_na_token(fs[j].b, fs[j].n) && !parse_double(fs[j].b, fs[j].n, d))
          types[j] = kEnum;
    }
  }
  for (size_t j = 0; j < forced.size() && j < ncol; ++j)
    if (forced[j] >= 0) types[j] = forced[j];
  P->types = types;
  P->num.assign(ncol, {});
  P->codes.assign(ncol, {});
  for (size_t j = 0; j < ncol; ++j) {
    if (types[j] == kNumeric) P->num[j].assign(nl, NAN);
    else P->codes[j].assign(nl, -1);
  }
  // pass 1 (parallel): numbers + per-thread string dictionaries for enum columns
  nthreads = std::max(1, std::min<int>(nthreads, (int)std::max<size_t>(1, nl / 4096)));
  std::vector<std::vector<std::unordered_map<std::string, int32_t>>> local(nthreads,
                                                                           std::vector<std::unordered_map<std::string, int32_t>>(ncol));
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) {
    th.emplace_back([&, t] {
      std::vector<Field> fs;
      std::vector<std::string> scr;
      size_t lo = nl * t / nthreads, hi = nl * (t + 1) / nthreads;
      for (size_t i = lo; i < hi; ++i) {
        split_line(lines[start + i].first, lines[start + i].second, sep, fs, scr);
        for (size_t j = 0; j < ncol; ++j) {
          if (j >= fs.size() || is_na_token(fs[j].b, fs[j].n)) continue;
          if (types[j] == kNumeric) {
            double d;
            if (parse_double(fs[j].b, fs[j].n, d)) P->num[j][i] = d;
          } else {
            auto& dict = local[t][j];
            auto it = dict.emplace(std::string(fs[j].b, fs[j].n), (int32_t)dict.size()).first;
            P->codes[j][i] = it->second;  // thread-local code, remapped below
          }
        }
      }
    });
  }
  for (auto& x : th) x.join();
  // merge dictionaries into sorted domains, remap codes
  P->domains.assign(ncol, {});
  for (size_t j = 0; j < ncol; ++j) {
    if (types[j] == kNumeric) continue;
    std::map<std::string, int32_t> all;
    for (int t = 0; t < nthreads; ++t)
      for (auto& kv : local[t][j]) all.emplace(kv.first, 0);
    int32_t k = 0;
    for (auto& kv : all) {
      kv.second = k++;
      P->domains[j].push_back(kv.first);
    }
    std::vector<std::vector<int32_t>> remap(nthreads);
    for (int t = 0; t < nthreads; ++t) {
      remap[t].assign(local[t][j].size(), -1);
      for (auto& kv : local[t][j]) remap[t][kv.second] = all[kv.first];
    }
    for (int t = 0; t < nthreads; ++t) {
      size_t lo = nl * t / nthreads, hi = nl * (t + 1) / nthreads;
      for (size_t i = lo; i < hi; ++i) {
        int32_t c = P->codes[j][i];
        if (c >= 0) P->codes[j][i] = remap[t][c];
      }
    }
  }
  return P;
}

std::string read_range(const char* path, int64_t start, int64_t end, std::string& err) {
  std::ifstream in(path, std::ios::binary);
  if (!in) {
    err = std::string("cannot open ") + path;
    return "";
  }
  in.seekg(0, std::ios::end);
  int64_t size = in.tellg();
  if (end < 0 || end > size) end = size;
  if (start < 0) start = 0;
  // align the range to line boundaries: a shard starts after the first newline
  // at or past `start` (unless start == 0) and ends at the first newline at or
  // past `end`
  std::string data;
  if (start > 0) {
    // the line containing byte start-1 belongs to the previous shard
    int64_t p = start - 1;
    in.seekg(p);
    char c;
    while (in.get(c) && c != '\n') ++p;
    start = p + 1;
  }
  if (start >= size) return "";
  int64_t stop = end;
  if (end < size) {
    in.seekg(end - 1);
    char c;
    while (in.get(c) && c != '\n') ++stop;
  }
  if (stop > size) stop = size;
  data.resize((size_t)std::max<int64_t>(0, stop - start));
  in.seekg(start);
  in.read(&data[0], (std::streamsize)data.size());
  return data;
}

}  // namespace

H2OMX_HOST_API void* h2omx_csv_parse(const char* path, char sep, int header, int nthreads, int64_t start,
                                     int64_t end, const int* forced_types, int n_forced) {
  std::string err;
  std::string data = read_range(path, start, end, err);
  std::vector<int> forced(forced_types ? forced_types : nullptr, forced_types ? forced_types + n_forced : nullptr);
  if (!err.empty()) {
    auto* P = new Parsed();
    P->error = err;
    return P;
  }
  return parse_buffer(data, sep, header, nthreads, forced);
}

H2OMX_HOST_API void* h2omx_csv_parse_text(const char* text, int64_t len, char sep, int header, int nthreads) {
  std::string data(text, (size_t)len);
  return parse_buffer(data, sep, header, nthreads, {});
}

H2OMX_HOST_API const char* h2omx_csv_error(void* h) {
  auto* P = static_cast<Parsed*>(h);
  return P->error.empty() ? nullptr : P->error.c_str();
}
H2OMX_HOST_API int h2omx_csv_ncols(void* h) { return (int)static_cast<Parsed*>(h)->names.size(); }
H2OMX_HOST_API int64_t h2omx_csv_nrows(void* h) { return static_cast<Parsed*>(h)->nrows; }
H2OMX_HOST_API int h2omx_csv_header(void* h) { return static_cast<Parsed*>(h)->header; }
H2OMX_HOST_API char h2omx_csv_sep(void* h) { return static_cast<Parsed*>(h)->sep; }
H2OMX_HOST_API const char* h2omx_csv_colname(void* h, int j) { return static_cast<Parsed*>(h)->names[j].c_str(); }
H2OMX_HOST_API int h2omx_csv_coltype(void* h, int j) { return static_cast<Parsed*>(h)->types[j]; }
H2OMX_HOST_API int h2omx_csv_numeric(void* h, int j, double* out) {
  auto* P = static_cast<Parsed*>(h);
  if (P->types[j] != kNumeric) return 1;
  std::memcpy(out, P->num[j].data(), P->num[j].size() * sizeof(double));
  return 0;
}
H2OMX_HOST_API int h2omx_csv_codes(void* h, int j, int32_t* out) {
  auto* P = static_cast<Parsed*>(h);
  if (P->types[j] == kNumeric) return 1;
  std::memcpy(out, P->codes[j].data(), P->codes[j].size() * sizeof(int32_t));
  return 0;
}
H2OMX_HOST_API int h2omx_csv_domain_size(void* h, int j) { return (int)static_cast<Parsed*>(h)->domains[j].size(); }
H2OMX_HOST_API const char* h2omx_csv_domain(void* h, int j, int k) {
  return static_cast<Parsed*>(h)->domains[j][k].c_str();
}
H2OMX_HOST_API void h2omx_csv_free(void* h) { delete static_cast<Parsed*>(h); }

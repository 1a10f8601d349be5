// krcn_svmlight.hip — multithreaded native parser of LIBSVM / svmlight text
// (host code).
//
// Replaces the reference's dataset load, sklearn.datasets.load_svmlight_file
// (cubic_newton.py:52-53: its Cython loop, _svmlight_format_fast.pyx, walks
// the file line by line on one core).  Here the text is cut into T byte ranges
// at line boundaries, each range is parsed by its own thread into local
// arrays, and the ranges are stitched by prefix sums into one CSR.  The
// semantics are sklearn's, checked value for value in tests/test_libsvm.py:
//   * '#' starts a comment that runs to the end of the line; a line with no
//     token is skipped (no row); `label [qid:q] idx:value ...` otherwise;
//   * label and values are decimal floats parsed correctly rounded (Python's
//     float(): optional sign, exponent, inf / infinity / nan in any case);
//     indices are decimal integers with an optional sign;
//   * an index < 0 raises "Invalid index", an index <= the previous one of
//     the row raises "should be sorted and unique" (duplicates are an error
//     in sklearn, not summed);
//   * zero-based detection and the shift of one-based files happen in the
//     caller (krcn.libsvm), from the minimum index this parser reports.
#include "krcn_host.hpp"

#include <algorithm>
#include <charconv>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

struct krcn_svm {
  int64_t rows = 0, nnz = 0, max_index = -1, min_index = -1;
  std::vector<int64_t> indptr;   // rows + 1
  std::vector<int64_t> indices;
  std::vector<double> data, labels;
};

namespace {

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\f' || c == '\v'; }

// Python float() of one token [p, e): correctly rounded (std::from_chars; strtod
// for results out of range, which Python rounds to +-inf / +-0 as strtod does).
bool parse_float(const char* p, const char* e, double* out) {
  if (p == e) return false;
  const char* q = p;
  bool neg = false;
  if (*q == '+' || *q == '-') {
    neg = *q == '-';
    ++q;
  }
  if (q == e || *q == '+' || *q == '-') return false;
  for (const char* r = q; r < e; ++r)
    if (*r == 'x' || *r == 'X' || *r == '_') return false;   // no hex / digit separators here
  double v = 0.0;
  const auto res = std::from_chars(q, e, v, std::chars_format::general);
  if (res.ec == std::errc::result_out_of_range) {
    std::string tok(q, e);
    v = std::strtod(tok.c_str(), nullptr);
  } else if (res.ec != std::errc() || res.ptr != e) {
    return false;
  }
  *out = neg ? -v : v;
  return true;
}

bool parse_int(const char* p, const char* e, int64_t* out) {
  if (p == e) return false;
  bool neg = false;
  if (*p == '+' || *p == '-') {
    neg = *p == '-';
    ++p;
  }
  if (p == e) return false;
  int64_t v = 0;
  for (; p < e; ++p) {
    if (*p < '0' || *p > '9') return false;
    if (v > (int64_t(1) << 56)) return false;   // far past any int32 index
    v = v * 10 + (*p - '0');
  }
  *out = neg ? -v : v;
  return true;
}

struct Part {
  std::vector<int64_t> rowlen, indices;
  std::vector<double> data, labels;
  int64_t max_index = -1, min_index = -1;
  int64_t lines = 0;        // lines walked (the error's line, relative to the range, on failure)
  std::string err;
};

void parse_range(const char* b, const char* e, Part& P) {
  int64_t& line = P.lines;
  const char* p = b;
  while (p < e) {
    const char* eol = static_cast<const char*>(std::memchr(p, '\n', size_t(e - p)));
    if (!eol) eol = e;
    const char* hash = static_cast<const char*>(std::memchr(p, '#', size_t(eol - p)));
    const char* end = hash ? hash : eol;
    // tokens of [p, end)
    const char* t = p;
    while (t < end && is_space(*t)) ++t;
    if (t < end) {
      const char* te = t;
      while (te < end && !is_space(*te)) ++te;
      double label;
      if (!parse_float(t, te, &label)) {
        P.err = "@could not convert string to float: '" + std::string(t, te) + "'";
        return;
      }
      P.labels.push_back(label);
      int64_t prev = -1, count = 0;
      bool first_feature = true;
      t = te;
      for (;;) {
        while (t < end && is_space(*t)) ++t;
        if (t >= end) break;
        te = t;
        while (te < end && !is_space(*te)) ++te;
        const char* colon = static_cast<const char*>(std::memchr(t, ':', size_t(te - t)));
        if (first_feature && te - t >= 3 && t[0] == 'q' && t[1] == 'i' && t[2] == 'd') {
          first_feature = false;   // qid:<q> (sklearn: only the first token is checked)
          if (!colon) {
            P.err = "@not enough values to unpack in '" + std::string(t, te) + "'";
            return;
          }
          t = te;
          continue;
        }
        first_feature = false;
        if (!colon) {
          P.err = "@not enough values to unpack in '" + std::string(t, te) + "'";
          return;
        }
        int64_t idx;
        double val;
        if (!parse_int(t, colon, &idx)) {
          P.err = "@invalid literal for int() with base 10: '" +
                  std::string(t, colon) + "'";
          return;
        }
        if (idx < 0) {
          P.err = "Invalid index " + std::to_string(idx) + " in SVMlight/LibSVM data file.";
          return;
        }
        if (idx <= prev) {
          P.err = "Feature indices in SVMlight/LibSVM data file should be sorted and unique.";
          return;
        }
        if (!parse_float(colon + 1, te, &val)) {
          P.err = "@could not convert string to float: '" +
                  std::string(colon + 1, te) + "'";
          return;
        }
        P.indices.push_back(idx);
        P.data.push_back(val);
        P.max_index = std::max(P.max_index, idx);
        P.min_index = P.min_index < 0 ? idx : std::min(P.min_index, idx);
        prev = idx;
        ++count;
        t = te;
      }
      P.rowlen.push_back(count);
    }
    p = eol + 1;
    ++line;
  }
}

}  // namespace

extern "C" krcn_status krcn_svm_parse(const char* text, int64_t len, int threads, krcn_svm** out,
                                      int64_t* info4_host) {
  if (!out || !info4_host || (len > 0 && !text)) return fail(KRCN_ERR_INVALID, "krcn_svm_parse: null argument");
  *out = nullptr;
  if (len < 0) return fail(KRCN_ERR_INVALID, "krcn_svm_parse: negative length");
  int T = threads > 0 ? threads : int(std::thread::hardware_concurrency());
  T = std::max(1, std::min(T, 64));
  if (len < (int64_t(1) << 20)) T = 1;   // small inputs: one range
  // range starts at line boundaries
  std::vector<int64_t> cut(T + 1, len);
  cut[0] = 0;
  for (int k = 1; k < T; ++k) {
    int64_t c = std::max(cut[k - 1], len * k / T);
    while (c < len && c > 0 && text[c - 1] != '\n') ++c;
    cut[k] = c;
  }
  std::vector<Part> parts(T);
  {
    std::vector<std::thread> th;
    for (int k = 1; k < T; ++k)
      th.emplace_back(parse_range, text + cut[k], text + cut[k + 1], std::ref(parts[k]));
    parse_range(text + cut[0], text + cut[1], parts[0]);
    for (auto& t : th) t.join();
  }
  int64_t line0 = 1;   // the failing line's number: lines of the ranges before it + its own
  for (const Part& P : parts) {
    if (!P.err.empty()) {
      if (P.err[0] == '@')
        return fail(KRCN_ERR_INVALID, "line %lld: %s", (long long)(line0 + P.lines), P.err.c_str() + 1);
      return fail(KRCN_ERR_INVALID, "%s", P.err.c_str());
    }
    line0 += P.lines;
  }
  krcn_svm* r = new krcn_svm();
  int64_t rows = 0, nnz = 0;
  for (const Part& P : parts) {
    rows += int64_t(P.rowlen.size());
    nnz += int64_t(P.indices.size());
    r->max_index = std::max(r->max_index, P.max_index);
    if (P.min_index >= 0) r->min_index = r->min_index < 0 ? P.min_index : std::min(r->min_index, P.min_index);
  }
  r->rows = rows;
  r->nnz = nnz;
  r->indptr.resize(size_t(rows) + 1);
  r->indices.resize(size_t(nnz));
  r->data.resize(size_t(nnz));
  r->labels.resize(size_t(rows));
  std::vector<int64_t> row0(T + 1, 0), nz0(T + 1, 0);
  for (int k = 0; k < T; ++k) {
    row0[k + 1] = row0[k] + int64_t(parts[k].rowlen.size());
    nz0[k + 1] = nz0[k] + int64_t(parts[k].indices.size());
  }
  r->indptr[0] = 0;
  {
    auto stitch = [&](int k) {
      const Part& P = parts[k];
      int64_t acc = nz0[k];
      for (size_t i = 0; i < P.rowlen.size(); ++i) {
        acc += P.rowlen[i];
        r->indptr[size_t(row0[k]) + i + 1] = acc;
      }
      std::copy(P.indices.begin(), P.indices.end(), r->indices.begin() + nz0[k]);
      std::copy(P.data.begin(), P.data.end(), r->data.begin() + nz0[k]);
      std::copy(P.labels.begin(), P.labels.end(), r->labels.begin() + row0[k]);
    };
    std::vector<std::thread> th;
    for (int k = 1; k < T; ++k) th.emplace_back(stitch, k);
    stitch(0);
    for (auto& t : th) t.join();
  }
  info4_host[0] = rows;
  info4_host[1] = nnz;
  info4_host[2] = r->max_index;
  info4_host[3] = r->min_index;
  *out = r;
  return KRCN_OK;
}

extern "C" krcn_status krcn_svm_export(const krcn_svm* p, int64_t shift, int32_t* indptr, int32_t* indices,
                                       double* data, double* labels) {
  if (!p || !indptr || (p->nnz && (!indices || !data)) || (p->rows && !labels))
    return fail(KRCN_ERR_INVALID, "krcn_svm_export: null argument");
  if (p->nnz >= (int64_t(1) << 31) || p->max_index - shift >= (int64_t(1) << 31))
    return fail(KRCN_ERR_UNSUPPORTED, "krcn_svm_export: int32 CSR needs nnz and indices < 2^31");
  if (shift != 0 && p->min_index >= 0 && p->min_index < shift)
    return fail(KRCN_ERR_INVALID, "krcn_svm_export: shift %lld past the smallest index %lld", (long long)shift,
                (long long)p->min_index);
  for (int64_t i = 0; i <= p->rows; ++i) indptr[i] = int32_t(p->indptr[size_t(i)]);
  for (int64_t e = 0; e < p->nnz; ++e) indices[e] = int32_t(p->indices[size_t(e)] - shift);
  if (p->nnz) std::memcpy(data, p->data.data(), sizeof(double) * size_t(p->nnz));
  if (p->rows) std::memcpy(labels, p->labels.data(), sizeof(double) * size_t(p->rows));
  return KRCN_OK;
}

extern "C" krcn_status krcn_svm_destroy(krcn_svm* p) {
  delete p;
  return KRCN_OK;
}

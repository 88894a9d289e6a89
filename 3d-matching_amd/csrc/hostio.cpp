// hostio.cpp — host-side helpers of the PLY/STL I/O in m3d.plyio:
// ASCII number blocks and the STL vertex merge.  The reference reads PLY through Open3D (o3d.io.read_point_cloud, src/ply/ply.py:80)
// and writes the converted cloud through trimesh (convert_stl-ply.py:1-11, encoding="ascii"),
// both compiled code; numpy's text paths (loadtxt / savetxt) cost ~1–3 µs per number.  Parsing
// uses std::from_chars (correctly rounded, the same doubles numpy's parser returns), formatting
// std::to_chars (the shortest representation that reads back to the same double).
#include <immintrin.h>
#include <charconv>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <system_error>
#include <vector>
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <limits>
#include <mutex>
#include <thread>

#include "../../include/m3d.h"

namespace {
inline bool is_blank(char c) { return c == ' ' || c == '\t' || c == '\r'; }

// threads of the text helpers: min(16, hardware threads, M3D_HOST_THREADS if set)
int host_threads() {
  static const int t = [] {
    int v = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    if (const char* e = getenv("M3D_HOST_THREADS")) v = std::max(1, std::min(v, atoi(e)));
    return v;
  }();
  return t;
}

// Exact fast path for the plain decimals of point files: [-]digits[.digits][(e|E)[±]digits]
// with at most 19 significant digits w and a decimal exponent |q| ≤ 27.  w and 10^|q| are exact
// in the x87 80-bit format (64-bit significand; 5^27 < 2^64), so w·10^q (or w / 10^−q) is ONE
// correctly rounded extended-precision operation; converting that to double is a second
// rounding, which can differ from the correctly rounded double only when the extended result
// lies within one extended ulp of a point halfway between two doubles (its low 11 significand
// bits 0x3FF–0x401) — those, and everything outside the form, return nullptr and take
// std::from_chars.  Results in this range are normal doubles (|x| in [1e-27, 1e46]).
const long double kPow10L[28] = {1e0L,  1e1L,  1e2L,  1e3L,  1e4L,  1e5L,  1e6L,  1e7L,  1e8L,  1e9L,
                                 1e10L, 1e11L, 1e12L, 1e13L, 1e14L, 1e15L, 1e16L, 1e17L, 1e18L, 1e19L,
                                 1e20L, 1e21L, 1e22L, 1e23L, 1e24L, 1e25L, 1e26L, 1e27L};

// The fast path needs the x87 format (64-bit significand stored first) AND the FPU running at
// extended precision: compiled out where long double is anything else (IEEE quad, plain
// double), switched off at run time when the precision-control word rounds to 53 bits.
constexpr bool kX87Long = std::numeric_limits<long double>::digits == 64 &&
                          std::numeric_limits<long double>::radix == 2;

bool x87_extended_active() {
  static const bool ok = [] {
    volatile long double one = 1.0L, tiny = 1.0L;
    for (int i = 0; i < 63; ++i) tiny = tiny / 2.0L;  // 2^-63: representable only at 64 bits
    return kX87Long && (long double)(one + tiny) != one;
  }();
  return ok;
}

inline const char* parse_decimal_fast(const char* p, const char* e, double* out) {
  if constexpr (!kX87Long) {
    return nullptr;
  }
  if (!x87_extended_active()) return nullptr;
  const char* s = p;
  const bool neg = s < e && *s == '-';
  s += neg;
  // w < 10^18 before each digit keeps w < 10^19 < 2^64: at most 19 significant digits
  constexpr uint64_t kW18 = 1000000000000000000ull;
  uint64_t w = 0;
  int q = 0;
  const char* const ds = s;
  while (s < e && (unsigned)(*s - '0') < 10) {
    if (w >= kW18) return nullptr;
    w = w * 10 + (unsigned)(*s++ - '0');
  }
  bool any = s > ds;
  if (s < e && *s == '.') {
    const char* const fs = ++s;
    while (s < e && (unsigned)(*s - '0') < 10) {
      if (w >= kW18) return nullptr;
      w = w * 10 + (unsigned)(*s++ - '0');
    }
    q = -(int)(s - fs);
    any |= s > fs;
  }
  if (!any) return nullptr;
  if (s < e && (*s == 'e' || *s == 'E')) {
    ++s;
    bool eneg = false;
    if (s < e && (*s == '-' || *s == '+')) eneg = *s++ == '-';
    int x = 0, xd = 0;
    while (s < e && (unsigned)(*s - '0') < 10 && xd < 5) x = x * 10 + (*s++ - '0'), ++xd;
    if (xd == 0 || xd == 5) return nullptr;
    q += eneg ? -x : x;
  }
  double v;
  if (w == 0) {
    v = 0.0;
  } else if (q == 0) {
    v = (double)w;  // one correctly rounded conversion
  } else {
    if (q > 27 || q < -27) return nullptr;
    const long double L = q > 0 ? (long double)w * kPow10L[q] : (long double)w / kPow10L[-q];
    uint64_t m;
    memcpy(&m, &L, sizeof(m));  // x87 extended: the 64-bit significand comes first
    const uint64_t lo = m & 0x7FF;
    if (lo >= 0x3FF && lo <= 0x401) return nullptr;
    v = (double)L;
  }
  *out = neg ? -v : v;
  return s;
}
}  // namespace

extern "C" {

namespace {
// serial parse of `rows` rows from [buf, buf + len): the rows' numbers into out, *consumed = bytes
// up to and including the last row's newline
int parse_rows_serial(const char* buf, size_t len, int64_t rows, int32_t cols, double* out,
                      size_t* consumed) {
  const char* p = buf;
  const char* const e = buf + len;
  int64_t r = 0;
  while (r < rows) {
    if (p >= e) return M3D_ERR_INVALID;  // fewer rows than declared
    int32_t c = 0;
    for (;;) {
      while (p < e && is_blank(*p)) ++p;
      if (p >= e || *p == '\n') break;
      if (c == cols) return M3D_ERR_INVALID;  // more numbers on the row than properties
      double v;
      const char* end = parse_decimal_fast(p, e, &v);
      if (end == nullptr) {
        const std::from_chars_result res = std::from_chars(p, e, v);
        if (res.ec != std::errc()) return M3D_ERR_INVALID;
        end = res.ptr;
      }
      if (end < e && !is_blank(*end) && *end != '\n')
        return M3D_ERR_INVALID;  // not a plain number (the caller falls back to numpy)
      out[r * cols + c++] = v;
      p = end;
    }
    if (p < e) ++p;  // the newline
    if (c == 0) continue;  // blank line
    if (c != cols) return M3D_ERR_INVALID;
    ++r;
  }
  *consumed = (size_t)(p - buf);
  return M3D_OK;
}

// rows (lines holding anything but blanks) in [b, e): the serial parser's row rule
int64_t count_rows(const char* b, const char* e) {
  int64_t n = 0;
  bool any = false;
  for (const char* p = b; p < e; ++p) {
    const char c = *p;
    if (c == '\n') {
      n += any;
      any = false;
    } else {
      any |= !is_blank(c);
    }
  }
  return n + any;
}
}  // namespace

// Large inputs are parsed by several threads: the buffer is cut into chunks at line starts, each
// thread counts its chunk's rows, the prefix sums place every chunk's rows in `out` (and find the
// chunk holding the last row to parse), then the chunks are parsed in parallel.  (The fast
// decimal path scales across threads; std::from_chars of this libstdc++ hardly does.)
int m3d_parse_ascii_rows(const char* buf, size_t len, int64_t rows, int32_t cols, double* out,
                         size_t* consumed) {
  if ((len > 0 && buf == nullptr) || rows < 0 || cols <= 0 || (rows > 0 && out == nullptr) ||
      consumed == nullptr)
    return M3D_ERR_INVALID;
  const int T = (int)std::min<size_t>((size_t)host_threads(), len / ((size_t)1 << 18));
  if (T < 2 || rows < 4096) return parse_rows_serial(buf, len, rows, cols, out, consumed);
  std::vector<size_t> cut((size_t)T + 1, len);
  cut[0] = 0;
  for (int t = 1; t < T; ++t) {
    const size_t c = std::max(cut[t - 1], len / T * (size_t)t);
    const void* nl = c < len ? memchr(buf + c, '\n', len - c) : nullptr;
    cut[t] = nl ? (size_t)((const char*)nl - buf) + 1 : len;
  }
  std::vector<int64_t> nrow((size_t)T, 0);
  std::vector<int> rc((size_t)T, M3D_OK);
  std::vector<size_t> used((size_t)T, 0);
  auto run = [&](auto&& body) {
    std::vector<std::thread> th;
    th.reserve((size_t)T - 1);
    for (int t = 1; t < T; ++t) th.emplace_back(body, t);
    body(0);
    for (auto& x : th) x.join();
  };
  run([&](int t) { nrow[t] = count_rows(buf + cut[t], buf + cut[t + 1]); });
  std::vector<int64_t> first((size_t)T + 1, 0);
  for (int t = 0; t < T; ++t) first[t + 1] = first[t] + nrow[t];
  if (first[T] < rows) return M3D_ERR_INVALID;  // fewer rows than declared
  run([&](int t) {
    const int64_t want = std::min(nrow[t], rows - first[t]);
    if (want <= 0) return;
    rc[t] = parse_rows_serial(buf + cut[t], cut[t + 1] - cut[t], want, cols, out + first[t] * cols,
                              &used[t]);
  });
  int last = 0;
  for (int t = 0; t < T; ++t) {
    if (rc[t] != M3D_OK) return rc[t];
    if (first[t] < rows) last = t;
  }
  *consumed = cut[last] + used[last];
  return M3D_OK;
}

namespace {
// rows [r0, r1) as text into [p, e): nullptr if it does not fit
char* format_rows(const double* data, int64_t r0, int64_t r1, int32_t cols, char* p, char* e) {
  for (int64_t r = r0; r < r1; ++r)
    for (int32_t c = 0; c < cols; ++c) {
      if (e - p < 32) return nullptr;  // a double takes at most 24 characters
      const std::to_chars_result res = std::to_chars(p, e, data[r * cols + c]);
      if (res.ec != std::errc()) return nullptr;
      p = res.ptr;
      *p++ = (c + 1 < cols) ? ' ' : '\n';
    }
  return p;
}
}  // namespace

// Large blocks are formatted by several threads into their own buffers (std::to_chars is
// locale-free), then copied into `out` in row order.
int m3d_format_ascii_rows(const double* data, int64_t rows, int32_t cols, char* out, size_t cap,
                          size_t* written) {
  if (rows < 0 || cols <= 0 || (rows > 0 && (data == nullptr || out == nullptr)) || written == nullptr)
    return M3D_ERR_INVALID;
  const int T = (int)std::min<int64_t>((int64_t)host_threads(), rows * cols / 32768);
  if (T < 2) {
    char* p = format_rows(data, 0, rows, cols, out, out + cap);
    if (p == nullptr) return M3D_ERR_INVALID;
    *written = (size_t)(p - out);
    return M3D_OK;
  }
  std::vector<std::vector<char>> part((size_t)T);
  std::vector<size_t> len((size_t)T, 0);
  std::vector<int> ok((size_t)T, 1);
  auto body = [&](int t) {
    const int64_t r0 = rows * t / T, r1 = rows * (t + 1) / T;
    part[t].resize((size_t)(r1 - r0) * (size_t)cols * 25 + 32);
    char* b = part[t].data();
    char* p = format_rows(data, r0, r1, cols, b, b + part[t].size());
    ok[t] = p != nullptr;
    len[t] = p ? (size_t)(p - b) : 0;
  };
  std::vector<std::thread> th;
  th.reserve((size_t)T - 1);
  for (int t = 1; t < T; ++t) th.emplace_back(body, t);
  body(0);
  for (auto& x : th) x.join();
  size_t total = 0;
  for (int t = 0; t < T; ++t) {
    if (!ok[t]) return M3D_ERR_INVALID;
    total += len[t];
  }
  if (total > cap) return M3D_ERR_INVALID;
  size_t off = 0;
  for (int t = 0; t < T; ++t) {
    memcpy(out + off, part[t].data(), len[t]);
    off += len[t];
  }
  *written = total;
  return M3D_OK;
}

// STL → unique vertices (convert_stl-ply.py: trimesh.load_mesh merges a mesh's shared
// corners).  Exact equality of the (x, y, z) bytes after -0.0 → +0.0, ids in first-occurrence
// order — what plyio's numpy sort-based merge computes, in one hash pass: open addressing over a
// power-of-two table of (32-bit hash tag, id) slots kept at ≤ 50 % load (it starts at n / 4
// slots — a closed mesh has ~n / 6 distinct corners — and doubles when half full), so the table
// stays cache-sized and a probe only reads the stored vertex when the tags agree; the slots of
// the vertices 8 ahead are prefetched.
namespace {
struct MergeSlot {
  uint32_t tag;
  int32_t id;  // −1: empty
};
inline uint64_t vertex_hash(const uint64_t b[3]) {
  uint64_t h = b[0] * 0x9E3779B97F4A7C15ull;
  h = (h ^ (h >> 29) ^ b[1]) * 0xBF58476D1CE4E5B9ull;
  h = (h ^ (h >> 31) ^ b[2]) * 0x94D049BB133111EBull;
  return h ^ (h >> 32);
}
inline void vertex_bits(const double* xyz, double v[3], uint64_t b[3]) {
  for (int k = 0; k < 3; ++k) {
    v[k] = xyz[k] + 0.0;  // -0.0 + 0.0 = +0.0
    memcpy(&b[k], &v[k], 8);
  }
}
}  // namespace

int m3d_merge_vertices(const double* xyz, int64_t n, double* uniq, int32_t* inverse,
                       int64_t* n_unique) {
  if (n < 0 || n > INT32_MAX || (n > 0 && (xyz == nullptr || uniq == nullptr || inverse == nullptr)) ||
      n_unique == nullptr)
    return M3D_ERR_INVALID;
  uint64_t cap = 1024;
  while (cap < (uint64_t)n / 4) cap <<= 1;
  std::vector<MergeSlot> table(cap, MergeSlot{0u, -1});
  std::vector<uint64_t> hashes;  // only for rehashing: the hash of each unique vertex
  hashes.reserve((size_t)(cap / 2));
  constexpr int64_t kAhead = 8;
  uint64_t hq[kAhead];  // hashes of vertices i .. i + kAhead − 1 (ring)
  for (int64_t i = 0; i < std::min<int64_t>(n, kAhead); ++i) {
    double v[3];
    uint64_t b[3];
    vertex_bits(xyz + 3 * i, v, b);
    hq[i] = vertex_hash(b);
    __builtin_prefetch(&table[hq[i] & (cap - 1)]);
  }
  int64_t m = 0;
  for (int64_t i = 0; i < n; ++i) {
    double v[3];
    uint64_t b[3];
    vertex_bits(xyz + 3 * i, v, b);
    const uint64_t h = hq[i % kAhead];
    if (i + kAhead < n) {
      double v2[3];
      uint64_t b2[3];
      vertex_bits(xyz + 3 * (i + kAhead), v2, b2);
      const uint64_t h2 = vertex_hash(b2);
      hq[i % kAhead] = h2;
      __builtin_prefetch(&table[h2 & (cap - 1)]);
    }
    const uint32_t tag = (uint32_t)(h >> 32);
    uint64_t s = h & (cap - 1);
    for (;;) {
      const MergeSlot e = table[s];
      if (e.id < 0) {
        table[s] = MergeSlot{tag, (int32_t)m};
        memcpy(uniq + 3 * m, v, sizeof(v));
        hashes.push_back(h);
        inverse[i] = (int32_t)m;
        ++m;
        if ((uint64_t)m * 2 > cap) {  // grow: reinsert every unique vertex by its stored hash
          cap <<= 1;
          std::vector<MergeSlot> t2(cap, MergeSlot{0u, -1});
          for (int64_t u = 0; u < m; ++u) {
            uint64_t s2 = hashes[(size_t)u] & (cap - 1);
            while (t2[s2].id >= 0) s2 = (s2 + 1) & (cap - 1);
            t2[s2] = MergeSlot{(uint32_t)(hashes[(size_t)u] >> 32), (int32_t)u};
          }
          table.swap(t2);
        }
        break;
      }
      if (e.tag == tag && memcmp(uniq + 3 * (int64_t)e.id, v, sizeof(v)) == 0) {
        inverse[i] = e.id;
        break;
      }
      s = (s + 1) & (cap - 1);
    }
  }
  *n_unique = m;
  return M3D_OK;
}

// Content keys of the drop-in's cache (m3d.cache "content" policy): the reference's per-call API
// (ransac.py:195-236 per hypothesis) hands the same arrays over again and again, and the cache
// must notice any in-place edit, so every call keys each array by its full content.  At Nc = 1e5
// that is ~5.6 MB per call; one thread of xxh3 took ~0.11 ms of a 0.15 ms call.  Here the arrays
// are cut into 64 KB chunks hashed by a persistent pool with XXH3-128 (Y. Collet's published
// algorithm, long-input path with the default secret; known-answer tested against the python
// xxhash package), then each array's chunk digests, its byte length and chunk count are hashed
// again with XXH3-128 into its 128-bit key; the result does not depend on the thread count.
// What "128-bit" buys: XXH3-128 is a NON-cryptographic 128-bit hash, so two different arrays of
// one length share a key with probability ≈ 2⁻¹²⁸ per pair of unrelated contents (round 3 chained
// 64-bit chunk digests, which bounded the key at 2⁻⁶⁴); it is no defence against a caller who
// crafts collisions on purpose.  Round 3 used XXH64 per chunk (kept below for its known answers).
namespace {
constexpr uint64_t kP1 = 11400714785074694791ull, kP2 = 14029467366897019727ull,
                   kP3 = 1609587929392839161ull, kP4 = 9650029242287828579ull,
                   kP5 = 2870177450012600261ull;
inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t rd64(const uint8_t* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}
inline uint64_t xx_round(uint64_t acc, uint64_t in) { return rotl64(acc + in * kP2, 31) * kP1; }
inline uint64_t xx_merge(uint64_t acc, uint64_t v) { return (acc ^ xx_round(0, v)) * kP1 + kP4; }

uint64_t xxh64(const uint8_t* p, size_t len, uint64_t seed) {
  const uint8_t* const end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + kP1 + kP2, v2 = seed + kP2, v3 = seed, v4 = seed - kP1;
    const uint8_t* const limit = end - 32;
    do {
      v1 = xx_round(v1, rd64(p));
      v2 = xx_round(v2, rd64(p + 8));
      v3 = xx_round(v3, rd64(p + 16));
      v4 = xx_round(v4, rd64(p + 24));
      p += 32;
    } while (p <= limit);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xx_merge(xx_merge(xx_merge(xx_merge(h, v1), v2), v3), v4);
  } else {
    h = seed + kP5;
  }
  h += (uint64_t)len;
  for (; p + 8 <= end; p += 8) h = rotl64(h ^ xx_round(0, rd64(p)), 27) * kP1 + kP4;
  if (p + 4 <= end) {
    uint32_t w;
    memcpy(&w, p, 4);
    h = rotl64(h ^ ((uint64_t)w * kP1), 23) * kP2 + kP3;
    p += 4;
  }
  for (; p < end; ++p) h = rotl64(h ^ ((uint64_t)*p * kP5), 11) * kP1;
  h ^= h >> 33;
  h *= kP2;
  h ^= h >> 29;
  h *= kP3;
  h ^= h >> 32;
  return h;
}

// ---- XXH3-128, inputs of at least 240 bytes (XXH3_hashLong_128b with the default secret, seed 0)
constexpr uint64_t kQ1 = 0x9E3779B185EBCA87ull, kQ2 = 0xC2B2AE3D27D4EB4Full, kQ3 = 0x165667B19E3779F9ull,
                   kQ4 = 0x85EBCA77C2B2AE63ull, kQ5 = 0x27D4EB2F165667C5ull;
constexpr uint32_t kR1 = 0x9E3779B1u, kR2 = 0x85EBCA77u, kR3 = 0xC2B2AE3Du;
alignas(64) constexpr uint8_t kSecret[192] = {
    0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c, 0xf7, 0x21, 0xad, 0x1c,
    0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb, 0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f,
    0xcb, 0x79, 0xe6, 0x4e, 0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21,
    0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6, 0x81, 0x3a, 0x26, 0x4c,
    0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb, 0x88, 0xd0, 0x65, 0x8b, 0x1b, 0x53, 0x2e, 0xa3,
    0x71, 0x64, 0x48, 0x97, 0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8,
    0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7, 0xc7, 0x0b, 0x4f, 0x1d,
    0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31, 0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64,
    0xea, 0xc5, 0xac, 0x83, 0x34, 0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb,
    0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49, 0xd3, 0x16, 0x55, 0x26, 0x29, 0xd4, 0x68, 0x9e,
    0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc, 0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce,
    0x45, 0xcb, 0x3a, 0x8f, 0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e,
};
constexpr size_t kStripe = 64, kSecretSize = sizeof(kSecret), kStripesPerBlock = (kSecretSize - kStripe) / 8,
                 kBlock = kStripe * kStripesPerBlock;
constexpr size_t kXxh3Min = 241;  // the long path: inputs above 240 bytes

inline void xxh3_acc512(uint64_t* __restrict acc, const uint8_t* __restrict in, const uint8_t* __restrict key) {
  for (int i = 0; i < 8; ++i) {
    const uint64_t v = rd64(in + 8 * i), k = v ^ rd64(key + 8 * i);
    acc[i ^ 1] += v;
    acc[i] += (k & 0xFFFFFFFFull) * (k >> 32);
  }
}
inline void xxh3_scramble(uint64_t* acc, const uint8_t* key) {
  for (int i = 0; i < 8; ++i) {
    uint64_t a = acc[i];
    a ^= a >> 47;
    a ^= rd64(key + 8 * i);
    acc[i] = a * kR1;
  }
}
inline uint64_t mul128_fold64(uint64_t a, uint64_t b) {
  const unsigned __int128 m = (unsigned __int128)a * b;
  return (uint64_t)m ^ (uint64_t)(m >> 64);
}
inline uint64_t xxh3_avalanche(uint64_t h) {
  h ^= h >> 37;
  h *= 0x165667919E3779F9ull;
  return h ^ (h >> 32);
}
inline uint64_t xxh3_merge(const uint64_t* acc, const uint8_t* key, uint64_t start) {
  uint64_t r = start;
  for (int i = 0; i < 4; ++i) r += mul128_fold64(acc[2 * i] ^ rd64(key + 16 * i), acc[2 * i + 1] ^ rd64(key + 16 * i + 8));
  return xxh3_avalanche(r);
}

// The stripe loop of whole blocks, vectorised as xxhash's own SSE2 / AVX2 kernels do (the same
// arithmetic per 64-bit lane: acc[i ^ 1] += v, acc[i] += lo32(v ^ k) · hi32(v ^ k)); the scalar
// xxh3_acc512 handles the partial block and the last stripe.  AVX2 is chosen at run time.
__attribute__((target("avx2"))) void xxh3_blocks_avx2(uint64_t* acc, const uint8_t* p, size_t nb) {
  __m256i a[2] = {_mm256_load_si256(reinterpret_cast<const __m256i*>(acc)),
                  _mm256_load_si256(reinterpret_cast<const __m256i*>(acc + 4))};
  const __m256i prime = _mm256_set1_epi32((int)kR1);
  for (size_t b = 0; b < nb; ++b) {
    const uint8_t* blk = p + b * kBlock;
    for (size_t s = 0; s < kStripesPerBlock; ++s) {
      for (int i = 0; i < 2; ++i) {
        const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(blk + s * kStripe + 32 * i));
        const __m256i k = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(kSecret + 8 * s + 32 * i));
        const __m256i dk = _mm256_xor_si256(v, k);
        const __m256i prod = _mm256_mul_epu32(dk, _mm256_shuffle_epi32(dk, _MM_SHUFFLE(0, 3, 0, 1)));
        a[i] = _mm256_add_epi64(a[i], _mm256_add_epi64(prod, _mm256_shuffle_epi32(v, _MM_SHUFFLE(1, 0, 3, 2))));
      }
    }
    for (int i = 0; i < 2; ++i) {  // scramble: a ^= a >> 47; a ^= key; a *= PRIME32_1
      const __m256i k = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(kSecret + kSecretSize - kStripe + 32 * i));
      const __m256i x = _mm256_xor_si256(_mm256_xor_si256(a[i], _mm256_srli_epi64(a[i], 47)), k);
      const __m256i lo = _mm256_mul_epu32(x, prime);
      const __m256i hi = _mm256_mul_epu32(_mm256_srli_epi64(x, 32), prime);
      a[i] = _mm256_add_epi64(lo, _mm256_slli_epi64(hi, 32));
    }
  }
  _mm256_store_si256(reinterpret_cast<__m256i*>(acc), a[0]);
  _mm256_store_si256(reinterpret_cast<__m256i*>(acc + 4), a[1]);
}

void xxh3_blocks_sse2(uint64_t* acc, const uint8_t* p, size_t nb) {
  __m128i a[4];
  for (int i = 0; i < 4; ++i) a[i] = _mm_load_si128(reinterpret_cast<const __m128i*>(acc + 2 * i));
  const __m128i prime = _mm_set1_epi32((int)kR1);
  for (size_t b = 0; b < nb; ++b) {
    const uint8_t* blk = p + b * kBlock;
    for (size_t s = 0; s < kStripesPerBlock; ++s) {
      for (int i = 0; i < 4; ++i) {
        const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(blk + s * kStripe + 16 * i));
        const __m128i k = _mm_loadu_si128(reinterpret_cast<const __m128i*>(kSecret + 8 * s + 16 * i));
        const __m128i dk = _mm_xor_si128(v, k);
        const __m128i prod = _mm_mul_epu32(dk, _mm_shuffle_epi32(dk, _MM_SHUFFLE(0, 3, 0, 1)));
        a[i] = _mm_add_epi64(a[i], _mm_add_epi64(prod, _mm_shuffle_epi32(v, _MM_SHUFFLE(1, 0, 3, 2))));
      }
    }
    for (int i = 0; i < 4; ++i) {
      const __m128i k = _mm_loadu_si128(reinterpret_cast<const __m128i*>(kSecret + kSecretSize - kStripe + 16 * i));
      const __m128i x = _mm_xor_si128(_mm_xor_si128(a[i], _mm_srli_epi64(a[i], 47)), k);
      const __m128i lo = _mm_mul_epu32(x, prime);
      const __m128i hi = _mm_mul_epu32(_mm_srli_epi64(x, 32), prime);
      a[i] = _mm_add_epi64(lo, _mm_slli_epi64(hi, 32));
    }
  }
  for (int i = 0; i < 4; ++i) _mm_store_si128(reinterpret_cast<__m128i*>(acc + 2 * i), a[i]);
}

// out[0] = low 64 bits, out[1] = high 64 bits (xxhash's xxh3_128_intdigest = high << 64 | low)
void xxh3_128_long(const uint8_t* p, size_t len, uint64_t out[2]) {
  alignas(64) uint64_t acc[8] = {kR3, kQ1, kQ2, kQ3, kQ4, kR2, kQ5, kR1};
  const size_t nb = (len - 1) / kBlock;
  static const bool avx2 = __builtin_cpu_supports("avx2") && getenv("M3D_XXH3_SSE2") == nullptr;
  if (avx2)
    xxh3_blocks_avx2(acc, p, nb);
  else
    xxh3_blocks_sse2(acc, p, nb);
  const size_t ns = ((len - 1) - kBlock * nb) / kStripe;
  for (size_t s = 0; s < ns; ++s) xxh3_acc512(acc, p + nb * kBlock + s * kStripe, kSecret + 8 * s);
  xxh3_acc512(acc, p + len - kStripe, kSecret + kSecretSize - kStripe - 7);
  out[0] = xxh3_merge(acc, kSecret + 11, (uint64_t)len * kQ1);
  out[1] = xxh3_merge(acc, kSecret + kSecretSize - 64 - 11, ~((uint64_t)len * kQ2));
}

constexpr size_t kHashChunk = (size_t)1 << 16;

struct HashJob {
  const uint8_t* p;
  size_t len;
  uint64_t* out;  // 2 words
};

// a chunk's 128-bit digest: XXH3-128 of the chunk (> 240 bytes: every chunk of an array of at
// least 256 KB is — the last one absorbs a short tail, see m3d_content_keys), else of the chunk
// zero-padded to 256 bytes (only whole arrays below 241 bytes; the length is in the array key)
inline void chunk_digest(const HashJob& j) {
  if (j.len >= kXxh3Min) {
    xxh3_128_long(j.p, j.len, j.out);
  } else {
    alignas(16) uint8_t pad[256] = {};
    if (j.len > 0) memcpy(pad, j.p, j.len);
    xxh3_128_long(pad, sizeof(pad), j.out);
  }
}

// Persistent workers (created on first use): a batch of n items is handed out with one atomic
// counter; the caller works too and waits for the last item.  In-order form (host_pipeline): the
// caller also receives each item's completion in index order (e.g. to issue the DMA of a staged
// chunk as soon as it and every chunk before it are ready).
class WorkPool {
 public:
  static WorkPool& get() {
    static WorkPool* pool = new WorkPool();  // never destroyed: workers outlive static teardown
    return *pool;
  }
  void run(int64_t n, const std::function<void(int64_t)>& fn, const std::function<void(int64_t)>* in_order) {
    std::lock_guard<std::mutex> one(run_mu_);  // one batch at a time
    std::unique_ptr<std::atomic<uint8_t>[]> done(new std::atomic<uint8_t>[(size_t)std::max<int64_t>(n, 1)]);
    for (int64_t k = 0; k < n; ++k) done[k].store(0, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      n_ = n;
      done_ = done.get();
      next_.store(0);
      left_.store(n);
      ++gen_;
    }
    cv_.notify_all();
    if (in_order == nullptr) {
      work();
    } else {
      for (int64_t k = 0; k < n;) {
        if (done[k].load(std::memory_order_acquire)) {
          (*in_order)(k++);
          continue;
        }
        if (!take_one()) std::this_thread::yield();
      }
    }
    std::unique_lock<std::mutex> lk(mu_);
    // every item done AND every worker that joined this batch out of work(): the function and
    // the flags are the caller's and die with this call
    done_cv_.wait(lk, [&] { return left_.load() == 0 && active_ == 0; });
    fn_ = nullptr;
    done_ = nullptr;
  }

 private:
  WorkPool() {
    const int n = std::max(0, std::min(host_threads(), 8) - 1);
    for (int t = 0; t < n; ++t)
      std::thread([this] { loop(); }).detach();
  }
  bool take_one() {
    const int64_t k = next_.fetch_add(1);
    if (k >= n_) return false;
    (*fn_)(k);
    done_[k].store(1, std::memory_order_release);
    if (left_.fetch_sub(1) == 1) {
      std::lock_guard<std::mutex> lk(mu_);
      done_cv_.notify_all();
    }
    return true;
  }
  void work() {
    while (take_one()) {
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen && fn_ != nullptr; });
        seen = gen_;
        ++active_;
      }
      work();
      {
        std::lock_guard<std::mutex> lk(mu_);
        --active_;
      }
      done_cv_.notify_all();
    }
  }
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int64_t)>* fn_ = nullptr;
  std::atomic<uint8_t>* done_ = nullptr;
  int64_t n_ = 0;
  std::atomic<int64_t> next_{0}, left_{0};
  uint64_t gen_ = 0;
  int active_ = 0;  // workers inside work() for the current batch (guarded by mu_)
};
}  // namespace

extern "C++" {
namespace m3d {
void host_pipeline(int64_t n, const std::function<void(int64_t)>& fn, const std::function<void(int64_t)>& in_order) {
  if (n <= 0) return;
  if (host_threads() > 1 && n > 1) {
    WorkPool::get().run(n, fn, &in_order);
    return;
  }
  for (int64_t k = 0; k < n; ++k) {
    fn(k);
    in_order(k);
  }
}
}  // namespace m3d
}  // extern "C++"

uint64_t m3d_debug_xxh64(const void* p, size_t len, uint64_t seed) {
  return xxh64(static_cast<const uint8_t*>(p), len, seed);
}

int m3d_debug_xxh3_128(const void* p, size_t len, uint64_t* out2) {
  if (out2 == nullptr || (p == nullptr && len > 0) || len < kXxh3Min) return M3D_ERR_INVALID;
  xxh3_128_long(static_cast<const uint8_t*>(p), len, out2);
  return M3D_OK;
}

int m3d_content_keys(const void* const* bufs, const size_t* lens, int32_t n, uint64_t* keys) {
  if (n < 0 || (n > 0 && (bufs == nullptr || lens == nullptr || keys == nullptr))) return M3D_ERR_INVALID;
  // chunk c of an array = [c·64 KB, (c + 1)·64 KB), except that a last piece shorter than the
  // XXH3 long-path minimum joins the chunk before it; an empty array has one empty chunk
  auto nchunks = [](size_t len) -> size_t {
    if (len <= kHashChunk) return 1;
    const size_t full = len / kHashChunk, tail = len - full * kHashChunk;
    return (tail == 0 || tail < kXxh3Min) ? full : full + 1;
  };
  std::vector<size_t> first((size_t)n + 1, 0);
  for (int32_t i = 0; i < n; ++i) {
    if (lens[i] > 0 && bufs[i] == nullptr) return M3D_ERR_INVALID;
    first[(size_t)i + 1] = first[(size_t)i] + nchunks(lens[i]);
  }
  std::vector<uint64_t> ch(2 * first[(size_t)n]);
  std::vector<HashJob> jobs;
  jobs.reserve(first[(size_t)n]);
  for (int32_t i = 0; i < n; ++i) {
    const uint8_t* b = static_cast<const uint8_t*>(bufs[i]);
    const size_t nc = first[(size_t)i + 1] - first[(size_t)i];
    for (size_t c = 0; c < nc; ++c) {
      const size_t off = c * kHashChunk;
      const size_t len = (c + 1 == nc) ? lens[i] - off : kHashChunk;
      jobs.push_back(HashJob{b + off, len, &ch[2 * (first[(size_t)i] + c)]});
    }
  }
  if (jobs.size() >= 4 && host_threads() > 1) {
    const std::function<void(int64_t)> fn = [&](int64_t k) { chunk_digest(jobs[(size_t)k]); };
    WorkPool::get().run((int64_t)jobs.size(), fn, nullptr);
  } else {
    for (const HashJob& j : jobs) chunk_digest(j);
  }
  // the array key: XXH3-128 of (chunk digests ‖ byte length ‖ chunk count), zero-padded to at
  // least 256 bytes (an injective encoding: the digest count follows from the length)
  std::vector<uint64_t> msg;
  for (int32_t i = 0; i < n; ++i) {
    const size_t nc = first[(size_t)i + 1] - first[(size_t)i];
    msg.assign(std::max<size_t>(32, 2 * nc + 2), 0);
    std::copy(ch.begin() + 2 * first[(size_t)i], ch.begin() + 2 * first[(size_t)i + 1], msg.begin());
    msg[2 * nc] = (uint64_t)lens[i];
    msg[2 * nc + 1] = (uint64_t)nc;
    xxh3_128_long(reinterpret_cast<const uint8_t*>(msg.data()), 8 * msg.size(), keys + 2 * i);
  }
  return M3D_OK;
}

}  // extern "C"

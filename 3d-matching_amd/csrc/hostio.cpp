// hostio.cpp — host-side helpers of the PLY/STL I/O in m3d.plyio:
// ASCII number blocks and the STL vertex merge.  The reference reads PLY through Open3D (o3d.io.read_point_cloud, src/ply/ply.py:80)
// and writes the converted cloud through trimesh (convert_stl-ply.py:1-11, encoding="ascii"),
// both compiled code; numpy's text paths (loadtxt / savetxt) cost ~1–3 µs per number.  Parsing
// uses std::from_chars (correctly rounded, the same doubles numpy's parser returns), formatting
// std::to_chars (the shortest representation that reads back to the same double).
#include <charconv>
#include <cstdint>
#include <cstring>
#include <system_error>
#include <vector>
#include <algorithm>

#include "../../include/m3d.h"

namespace {
inline bool is_blank(char c) { return c == ' ' || c == '\t' || c == '\r'; }
}  // namespace

extern "C" {

int m3d_parse_ascii_rows(const char* buf, size_t len, int64_t rows, int32_t cols, double* out,
                         size_t* consumed) {
  if ((len > 0 && buf == nullptr) || rows < 0 || cols <= 0 || (rows > 0 && out == nullptr) ||
      consumed == nullptr)
    return M3D_ERR_INVALID;
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
      const std::from_chars_result res = std::from_chars(p, e, v);
      if (res.ec != std::errc() || (res.ptr < e && !is_blank(*res.ptr) && *res.ptr != '\n'))
        return M3D_ERR_INVALID;  // not a plain number (the caller falls back to numpy)
      out[r * cols + c++] = v;
      p = res.ptr;
    }
    if (p < e) ++p;  // the newline
    if (c == 0) continue;  // blank line
    if (c != cols) return M3D_ERR_INVALID;
    ++r;
  }
  *consumed = (size_t)(p - buf);
  return M3D_OK;
}

int m3d_format_ascii_rows(const double* data, int64_t rows, int32_t cols, char* out, size_t cap,
                          size_t* written) {
  if (rows < 0 || cols <= 0 || (rows > 0 && (data == nullptr || out == nullptr)) || written == nullptr)
    return M3D_ERR_INVALID;
  char* p = out;
  char* const e = out + cap;
  for (int64_t r = 0; r < rows; ++r)
    for (int32_t c = 0; c < cols; ++c) {
      if (e - p < 32) return M3D_ERR_INVALID;  // a double takes at most 24 characters
      const std::to_chars_result res = std::to_chars(p, e, data[r * cols + c]);
      if (res.ec != std::errc()) return M3D_ERR_INVALID;
      p = res.ptr;
      *p++ = (c + 1 < cols) ? ' ' : '\n';
    }
  *written = (size_t)(p - out);
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

}  // extern "C"

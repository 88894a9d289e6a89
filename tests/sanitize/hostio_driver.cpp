// Host-sanitizer driver for csrc/hostio.cpp (the C-ABI's host text I/O, STL merge and content
// keys).  Built twice by tests/test_hostio_sanitizers.py — AddressSanitizer + UBSan, and
// ThreadSanitizer — and run on the CPU: random and adversarial inputs through every entry point,
// results checked against the C library (strtod / printf round trips) or by construction.
// Exit code 0 = all checks passed; any sanitizer report aborts with a non-zero code.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/m3d.h"

static int fails = 0;
#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                           \
    }                                                                    \
  } while (0)

static uint64_t bits(double v) {
  uint64_t b;
  std::memcpy(&b, &v, 8);
  return b;
}

// a double printed in one of several formats the parser sees in point files
static std::string fmt(double v, int style) {
  char b[64];
  switch (style) {
    case 0: std::snprintf(b, sizeof b, "%.17g", v); break;
    case 1: std::snprintf(b, sizeof b, "%.6f", v); break;
    case 2: std::snprintf(b, sizeof b, "%.9e", v); break;
    case 3: std::snprintf(b, sizeof b, "%g", v); break;
    default: std::snprintf(b, sizeof b, "%.3E", v); break;
  }
  return b;
}

static double random_value(std::mt19937_64& g) {
  std::uniform_int_distribution<int> kind(0, 9);
  std::uniform_real_distribution<double> u(-1.0, 1.0);
  switch (kind(g)) {
    case 0: return 0.0;
    case 1: return -0.0;
    case 2: return std::ldexp(u(g), (int)(g() % 2000) - 1000);  // wide exponents (incl. subnormal)
    case 3: return (double)(int64_t)(g() % 2000001) - 1000000.0;  // integers
    case 4: return u(g) * 1e-30;
    case 5: return u(g) * 1e30;
    default: return u(g) * 100.0;  // point coordinates
  }
}

static void test_parse(std::mt19937_64& g, int64_t rows, int cols) {
  std::vector<double> want((size_t)(rows * cols));
  std::string text;
  for (int64_t r = 0; r < rows; ++r) {
    if (g() % 50 == 0) text += (g() % 2) ? "\n" : "  \t\r\n";  // blank lines are skipped
    for (int c = 0; c < cols; ++c) {
      const double v = random_value(g);
      const std::string s = fmt(v, (int)(g() % 5));
      want[(size_t)(r * cols + c)] = std::strtod(s.c_str(), nullptr);
      if (c > 0 || g() % 4 == 0) text += (g() % 3 == 0) ? "\t" : " ";
      text += s;
    }
    text += (g() % 10 == 0) ? " \r\n" : "\n";
  }
  const std::string tail = "3 0 1 2\n";  // face lines after the vertex block
  text += tail;
  std::vector<double> got((size_t)(rows * cols) + 1, -7.0);
  size_t used = 0;
  CHECK(m3d_parse_ascii_rows(text.data(), text.size(), rows, cols, got.data(), &used) == M3D_OK);
  CHECK(used == text.size() - tail.size());
  for (size_t i = 0; i < want.size(); ++i) CHECK(bits(got[i]) == bits(want[i]));
  CHECK(got.back() == -7.0);  // nothing written past rows × cols
}

static void test_parse_malformed(std::mt19937_64& g) {
  double out[64];
  size_t used = 0;
  const char* bad[] = {"1 2\n3\n", "1 2 3\n", "1 x\n2 3\n", "1 2\n3 4", "--1 2\n", "1e 2\n", "1..2 3\n",
                       "", "\n\n\n", "1 2\n3 4 5\n", ". 1\n"};
  const int64_t want_rows[] = {2, 1, 2, 2, 1, 1, 1, 1, 1, 2, 1};
  for (size_t k = 0; k < sizeof(bad) / sizeof(bad[0]); ++k) {
    const int rc = m3d_parse_ascii_rows(bad[k], std::strlen(bad[k]), want_rows[k], 2, out, &used);
    // "1 2\n3 4" (no final newline) is a valid 2-row block; every other case is refused
    if (k == 3) CHECK(rc == M3D_OK && out[3] == 4.0);
    else CHECK(rc == M3D_ERR_INVALID);
  }
  // random bytes: any return code, no out-of-bounds access
  for (int it = 0; it < 2000; ++it) {
    const size_t n = g() % 200;
    std::vector<char> buf(n);
    for (auto& ch : buf) ch = "0123456789.eE+- \t\r\nxn"[g() % 21];
    std::vector<double> o(4 * 3);
    (void)m3d_parse_ascii_rows(buf.data(), buf.size(), 4, 3, o.data(), &used);
  }
  CHECK(m3d_parse_ascii_rows(nullptr, 5, 1, 1, out, &used) == M3D_ERR_INVALID);
  CHECK(m3d_parse_ascii_rows("1\n", 2, 1, 0, out, &used) == M3D_ERR_INVALID);
}

static void test_format(std::mt19937_64& g, int64_t rows, int cols) {
  std::vector<double> v((size_t)(rows * cols));
  for (auto& x : v) x = random_value(g);
  const size_t cap = (size_t)(32 * rows * cols);
  std::vector<char> out(cap + 16, '#');
  size_t written = 0;
  CHECK(m3d_format_ascii_rows(v.data(), rows, cols, out.data(), cap, &written) == M3D_OK);
  CHECK(written <= cap);
  for (size_t i = cap; i < out.size(); ++i) CHECK(out[i] == '#');
  std::vector<double> back(v.size());
  size_t used = 0;
  CHECK(m3d_parse_ascii_rows(out.data(), written, rows, cols, back.data(), &used) == M3D_OK);
  for (size_t i = 0; i < v.size(); ++i) CHECK(bits(back[i]) == bits(v[i]));
  // a buffer too small is refused, never overrun
  if (rows * cols > 0) {
    std::vector<char> small(40, '#');
    const int rc = m3d_format_ascii_rows(v.data(), rows, cols, small.data(), 8, &written);
    CHECK(rc == M3D_ERR_INVALID);
    for (size_t i = 8; i < small.size(); ++i) CHECK(small[i] == '#');
  }
}

static void test_merge(std::mt19937_64& g, int64_t n) {
  const int64_t pool = std::max<int64_t>(1, n / 5);
  std::vector<double> base((size_t)(3 * pool));
  for (auto& x : base) x = (g() % 7 == 0) ? 0.0 : random_value(g);
  std::vector<double> xyz((size_t)(3 * n));
  for (int64_t i = 0; i < n; ++i) {
    const int64_t k = (int64_t)(g() % (uint64_t)pool);
    for (int a = 0; a < 3; ++a) {
      double x = base[(size_t)(3 * k + a)];
      if (x == 0.0 && g() % 2) x = -0.0;  // -0.0 ≡ +0.0
      xyz[(size_t)(3 * i + a)] = x;
    }
  }
  std::vector<double> uniq((size_t)(3 * n) + 3, -9.0);
  std::vector<int32_t> inv((size_t)n + 1, -5);
  int64_t m = -1;
  CHECK(m3d_merge_vertices(xyz.data(), n, uniq.data(), inv.data(), &m) == M3D_OK);
  CHECK(m >= 0 && m <= n && m <= pool);
  CHECK(inv[(size_t)n] == -5);
  int32_t next = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int32_t id = inv[(size_t)i];
    CHECK(id >= 0 && id < m);
    CHECK(id <= next);  // first-occurrence order
    if (id == next) ++next;
    for (int a = 0; a < 3; ++a) CHECK(uniq[(size_t)(3 * id + a)] == xyz[(size_t)(3 * i + a)]);
  }
  CHECK(next == m);
  // distinct ids hold distinct vertices
  for (int64_t u = 1; u < std::min<int64_t>(m, 200); ++u)
    CHECK(std::memcmp(&uniq[(size_t)(3 * u)], &uniq[(size_t)(3 * (u - 1))], 24) != 0);
}

static void test_hash(std::mt19937_64& g) {
  CHECK(m3d_debug_xxh64("", 0, 0) == 0xEF46DB3751D8E999ull);  // published XXH64 test vector
  // keys: deterministic, independent of concurrency, sensitive to every byte
  std::vector<std::vector<uint8_t>> bufs;
  const size_t lens[] = {0, 1, 31, 32, 65535, 65536, 65537, 1 << 20, 3 * (1 << 18) + 5};
  for (size_t l : lens) {
    std::vector<uint8_t> b(l);
    for (auto& x : b) x = (uint8_t)g();
    bufs.push_back(std::move(b));
  }
  const int n = (int)bufs.size();
  std::vector<const void*> ptrs(n);
  std::vector<size_t> ls(n);
  for (int i = 0; i < n; ++i) {
    ptrs[i] = bufs[i].data();
    ls[i] = bufs[i].size();
  }
  std::vector<uint64_t> k0(2 * n);
  CHECK(m3d_content_keys(ptrs.data(), ls.data(), n, k0.data()) == M3D_OK);
  std::vector<std::thread> th;
  std::vector<int> ok(8, 1);
  for (int t = 0; t < 8; ++t)
    th.emplace_back([&, t] {
      for (int rep = 0; rep < 20; ++rep) {
        std::vector<uint64_t> k(2 * n);
        if (m3d_content_keys(ptrs.data(), ls.data(), n, k.data()) != M3D_OK || k != k0) ok[t] = 0;
      }
    });
  for (auto& x : th) x.join();
  for (int t = 0; t < 8; ++t) CHECK(ok[t]);
  bufs[7][123457] ^= 1;  // one bit of one chunk
  std::vector<uint64_t> k1(2 * n);
  CHECK(m3d_content_keys(ptrs.data(), ls.data(), n, k1.data()) == M3D_OK);
  for (int i = 0; i < n; ++i) CHECK((k1[2 * i] != k0[2 * i]) == (i == 7));
}

int main() {
  std::mt19937_64 g(12345);
  for (int64_t rows : {0, 1, 7, 100, 5000}) test_parse(g, rows, 3);
  test_parse(g, 20000, 6);  // above the threaded-parse threshold (≥ 256 KiB, ≥ 4096 rows)
  test_parse_malformed(g);
  for (int64_t rows : {0, 1, 33, 4000}) test_format(g, rows, 3);
  test_format(g, 40000, 3);  // threaded formatting
  for (int64_t n : {0, 1, 2, 100, 5000, 300000}) test_merge(g, n);
  test_hash(g);
  std::printf("hostio sanitizer driver: %d failed checks\n", fails);
  return fails == 0 ? 0 : 1;
}

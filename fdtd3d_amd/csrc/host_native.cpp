// Host-side native runtime: topology optimiser, Yee ranges, DAT/BMP output.
#include "host_native.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>
#include <tuple>

namespace fdtd {

double halo_cost(const Int3& size, const Int3& topo) {
  double chunk[3];
  for (int a = 0; a < 3; ++a) chunk[a] = (double)size[a] / topo[a];
  double cost = 0;
  for (int a = 0; a < 3; ++a) {
    if (topo[a] <= 1) continue;
    double other = 1;
    for (int b = 0; b < 3; ++b)
      if (b != a) other *= chunk[b];
    cost += (topo[a] > 2 ? 2 : 1) * other;
  }
  return cost;
}

Int3 optimal_topology(const Int3& size, int p, const std::vector<int>& axes) {
  auto allowed = [&](int a) { return std::find(axes.begin(), axes.end(), a) != axes.end(); };
  Int3 best = {p, 1, 1};
  bool have = false;
  std::tuple<double, int, int, int, int> bestkey;
  // first pass: rank grids no finer than the cells; second: any rank grid
  for (int pass = 0; pass < 2 && !have; ++pass)
  for (int px = 1; px <= p; ++px) {
    if (p % px) continue;
    for (int py = 1; py <= p / px; ++py) {
      if ((p / px) % py) continue;
      int pz = p / (px * py);
      Int3 t = {px, py, pz};
      bool ok = true;
      for (int a = 0; a < 3; ++a)
        if ((t[a] > 1 && !allowed(a)) || (pass == 0 && t[a] > size[a])) ok = false;
      if (!ok) continue;
      int uneven = 0, nsplit = 0;
      for (int a = 0; a < 3; ++a) {
        uneven += size[a] % t[a];
        nsplit += t[a] > 1;
      }
      auto key = std::make_tuple(halo_cost(size, t), uneven, nsplit, -t[0], -t[1]);
      if (!have || key < bestkey) {
        bestkey = key;
        best = t;
        have = true;
      }
    }
  }
  return best;
}

void chunk_bounds(int n, int p, int coord, int& lo, int& hi) {
  const int core = n / p;
  lo = coord * core;
  hi = (coord == p - 1) ? n : lo + core;
}

void global_range(int comp, const Int3& size, const std::vector<int>& active, Int3& lo, Int3& hi) {
  // start / end diffs (reference YeeGridLayout.h:131-182)
  static const int start[6][3] = {{0, 1, 1}, {1, 0, 1}, {1, 1, 0}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
  static const int end[6][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 1, 1}, {1, 0, 1}, {1, 1, 0}};
  for (int a = 0; a < 3; ++a) {
    const bool act = std::find(active.begin(), active.end(), a) != active.end();
    lo[a] = act ? start[comp][a] : 0;
    hi[a] = size[a] - (act ? end[comp][a] : 0);
  }
}

std::string grid_file_name(long step, int rank, const std::string& name, const std::string& dir) {
  char buf[64];
  std::snprintf(buf, sizeof(buf), "current[%ld]_rank-%d_", step, rank);
  std::string base = dir.empty() ? std::string(buf) : dir + "/" + buf;
  return base + name;
}

bool write_dat(const std::string& path, const void* data, size_t bytes) {
  std::ofstream f(path, std::ios::binary);
  if (!f) return false;
  f.write((const char*)data, (std::streamsize)bytes);
  return (bool)f;
}

namespace {
void put16(std::vector<unsigned char>& b, uint16_t v) {
  b.push_back(v & 0xff);
  b.push_back(v >> 8);
}
void put32(std::vector<unsigned char>& b, uint32_t v) {
  for (int i = 0; i < 4; ++i) b.push_back((v >> (8 * i)) & 0xff);
}
}  // namespace

bool write_bmp(const std::string& path, const std::vector<double>& v, int w, int h, const std::string& palette) {
  double vmin = std::numeric_limits<double>::infinity(), vmax = -vmin;
  for (double x : v) {
    vmin = std::min(vmin, x);
    vmax = std::max(vmax, x);
  }
  const double rng = vmax - vmin, half = rng / 2;
  const int row = (w * 3 + 3) & ~3;
  std::vector<unsigned char> img((size_t)row * h, 0);
  for (int y = 0; y < h; ++y) {
    unsigned char* r = &img[(size_t)(h - 1 - y) * row];  // bottom-up rows
    for (int x = 0; x < w; ++x) {
      const double val = v[(size_t)x * h + y] - vmin;
      unsigned char R, G, B;
      if (palette == "gray") {
        const unsigned char g = rng == 0 ? 0 : (unsigned char)std::min(255.0, val / rng * 255);
        R = G = B = g;
      } else if (rng != 0 && val > half) {  // reference palette, BMPHelper.cpp:61-95
        const double t = (val - half) / half;
        R = (unsigned char)(t * 255);
        G = (unsigned char)((1 - t) * 255);
        B = 0;
      } else {
        const double t = rng == 0 ? 0 : val / half;
        R = 0;
        G = (unsigned char)(t * 255);
        B = (unsigned char)((1 - t) * 255);
      }
      r[3 * x] = B;
      r[3 * x + 1] = G;
      r[3 * x + 2] = R;
    }
  }
  std::vector<unsigned char> hdr;
  hdr.push_back('B');
  hdr.push_back('M');
  put32(hdr, 54 + (uint32_t)img.size());
  put16(hdr, 0);
  put16(hdr, 0);
  put32(hdr, 54);
  put32(hdr, 40);
  put32(hdr, (uint32_t)w);
  put32(hdr, (uint32_t)h);
  put16(hdr, 1);
  put16(hdr, 24);
  put32(hdr, 0);
  put32(hdr, (uint32_t)img.size());
  put32(hdr, 2835);
  put32(hdr, 2835);
  put32(hdr, 0);
  put32(hdr, 0);
  std::ofstream f(path, std::ios::binary);
  if (!f) return false;
  f.write((const char*)hdr.data(), hdr.size());
  f.write((const char*)img.data(), img.size());
  return (bool)f;
}

// ---- hybrid pass geometry ----
namespace {
bool empty6(const Box6& b) { return b[3] <= b[0] || b[4] <= b[1] || b[5] <= b[2]; }
Box6 and6(const Box6& a, const Box6& b) {
  Box6 r;
  for (int d = 0; d < 3; ++d) {
    r[d] = std::max(a[d], b[d]);
    r[3 + d] = std::min(a[3 + d], b[3 + d]);
  }
  return r;
}
}  // namespace

std::vector<Box6> box_minus6(const Box6& a, const Box6& b) {
  std::vector<Box6> out;
  const Box6 c = and6(a, b);
  if (empty6(c)) {
    if (!empty6(a)) out.push_back(a);
    return out;
  }
  Box6 rest = a;
  for (int d = 0; d < 3; ++d) {
    if (rest[d] < c[d]) {
      Box6 sl = rest;
      sl[3 + d] = c[d];
      out.push_back(sl);
    }
    if (c[3 + d] < rest[3 + d]) {
      Box6 sl = rest;
      sl[d] = c[3 + d];
      out.push_back(sl);
    }
    rest[d] = c[d];
    rest[3 + d] = c[3 + d];
  }
  return out;
}

bool hybrid_windows(const Box6& alloc, const Box6& K, const Box6& Dm, int T, const bool* act, const Int3& size,
                    std::vector<std::vector<Box6>>& shells, std::vector<Box6>& copy) {
  shells.assign(T, {});
  copy.clear();
  const bool cut = !empty6(Dm);
  for (int s = 0; s < T; ++s) {
    const int n = T - s;
    // the core shrunk by n on the sides inside the domain (a side on the
    // domain border has no shell beyond it)
    Box6 Kd = K;
    for (int d = 0; d < 3; ++d) {
      if (!act[d]) continue;
      if (Kd[d] > 0) Kd[d] += n;
      if (Kd[3 + d] < size[d]) Kd[3 + d] -= n;
    }
    if (empty6(Kd)) return false;
    shells[s] = box_minus6(alloc, Kd);
    if (cut) {
      Box6 g = Dm;
      for (int d = 0; d < 3; ++d)
        if (act[d]) {
          g[d] -= n;
          g[3 + d] += n;
        }
      const Box6 w = and6(g, Kd);
      if (!empty6(w)) shells[s].push_back(w);
    }
  }
  copy = box_minus6(alloc, K);
  if (cut) {
    const Box6 w = and6(Dm, alloc);
    if (!empty6(w)) copy.push_back(w);
  }
  return true;
}

}  // namespace fdtd

// C ABI used by the Python driver (models/blocking.py _hybrid_plan_m): the
// hybrid pass geometry of fdtd::hybrid_windows, flattened as
// [n_0, boxes of step 0 ..., ..., n_{T-1}, ..., n_copy, copy boxes ...] (six
// ints lo[3] hi[3] per box).  Returns the ints written, -1 when a step's core
// vanishes (no hybrid plan), -2 when `cap` is too small.
extern "C" __attribute__((visibility("default"))) int fdtd_hybrid_windows(const int* alloc, const int* K,
                                                                         const int* Dm, const int* size,
                                                                         const int* act, int T, int* out, int cap) {
  fdtd::Box6 a, k, dm;
  for (int q = 0; q < 6; ++q) {
    a[q] = alloc[q];
    k[q] = K[q];
    dm[q] = Dm[q];
  }
  const bool ac[3] = {act[0] != 0, act[1] != 0, act[2] != 0};
  std::vector<std::vector<fdtd::Box6>> shells;
  std::vector<fdtd::Box6> copy;
  if (T < 1 || !fdtd::hybrid_windows(a, k, dm, T, ac, {size[0], size[1], size[2]}, shells, copy)) return -1;
  int n = 0;
  auto put = [&](const std::vector<fdtd::Box6>& v) {
    if (n + 1 + 6 * (int)v.size() > cap) return false;
    out[n++] = (int)v.size();
    for (const auto& b : v)
      for (int q = 0; q < 6; ++q) out[n++] = b[q];
    return true;
  };
  for (const auto& v : shells)
    if (!put(v)) return -2;
  if (!put(copy)) return -2;
  return n;
}

// C ABI used by the Python parity tests
extern "C" __attribute__((visibility("default"))) void fdtd_optimal_topology(const int* size, int nprocs,
                                                                                const int* axes, int naxes,
                                                                                int* out) {
  fdtd::Int3 s = {size[0], size[1], size[2]};
  std::vector<int> ax(axes, axes + naxes);
  fdtd::Int3 t = fdtd::optimal_topology(s, nprocs, ax);
  for (int a = 0; a < 3; ++a) out[a] = t[a];
}

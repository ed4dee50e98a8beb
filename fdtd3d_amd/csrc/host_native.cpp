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

}  // namespace fdtd

// C ABI used by the Python parity tests
extern "C" __attribute__((visibility("default"))) void fdtd_optimal_topology(const int* size, int nprocs,
                                                                                const int* axes, int naxes,
                                                                                int* out) {
  fdtd::Int3 s = {size[0], size[1], size[2]};
  std::vector<int> ax(axes, axes + naxes);
  fdtd::Int3 t = fdtd::optimal_topology(s, nprocs, ax);
  for (int a = 0; a < 3; ++a) out[a] = t[a];
}

// Host-side native runtime pieces shared by the standalone driver:
// topology optimiser, Yee computation ranges, DAT/BMP writers.
#pragma once

#include <array>
#include <cstdint>
#include <string>
#include <vector>

namespace fdtd {

using Int3 = std::array<int, 3>;

// ---- topology (same cost model as fdtd3d_amd/parallel/topology.py) ----
double halo_cost(const Int3& size, const Int3& topo);
Int3 optimal_topology(const Int3& size, int nprocs, const std::vector<int>& axes);
void chunk_bounds(int n, int p, int coord, int& lo, int& hi);

// ---- Yee layout (fdtd3d_amd/layout/yee.py) ----
// component index: 0..2 = Ex,Ey,Ez; 3..5 = Hx,Hy,Hz
void global_range(int comp, const Int3& size, const std::vector<int>& active_axes, Int3& lo, Int3& hi);

// ---- hybrid pass geometry (one plan for both drivers) ----
// A hybrid pass (models/blocking.py _init_hybrid) advances the core box K by
// T steps in the blocked kernel and steps the rest; step s (0-based) of the
// stepped shell covers everything of the allocated box but the core cells
// deeper than T - s inside K (depth along the active axes; a side of K on the
// domain border has no shell beyond it), plus the cut box Dm (a stepped
// dispersive box inside K; empty: none) grown by T - s; after the pass the
// shell (alloc minus K, plus Dm) is copied into the core pass's output.
// Boxes are lo[3], hi[3].  False when a step's core vanishes.
using Box6 = std::array<int, 6>;
std::vector<Box6> box_minus6(const Box6& a, const Box6& b);  // non-empty slabs: x low / high, y, z
bool hybrid_windows(const Box6& alloc, const Box6& K, const Box6& Dm, int T, const bool* act, const Int3& size,
                    std::vector<std::vector<Box6>>& shells, std::vector<Box6>& copy);

// ---- files (reference naming, Source/File-Management/Commons.h:56-68) ----
std::string grid_file_name(long step, int rank, const std::string& name, const std::string& dir);
bool write_dat(const std::string& path, const void* data, size_t bytes);
// rgb: "rgb" (blue-green-red) or "gray"; values row-major [w][h]; pixel (x, y), y = 0 top
bool write_bmp(const std::string& path, const std::vector<double>& values, int w, int h,
               const std::string& palette);

}  // namespace fdtd

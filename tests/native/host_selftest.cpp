// Host-runtime self test, built with AddressSanitizer + UndefinedBehaviorSanitizer
// by tests/test_native_cpu.py::test_host_runtime_under_sanitizers (the
// reference's only guards were ASSERT + backtrace, Source/Helpers/Assert.h:25-91).
// Exercises the settings parser (every option kind, cmd-file round trip, bad
// input), the topology optimiser, chunk bounds, file naming and the DAT / BMP
// writers; exits non-zero on the first failed check.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "host_native.h"
#include "settings_native.h"

static int g_fail = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                    \
    }                                                              \
  } while (0)

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : ".";
  {
    fdtd::Settings s;
    const char* a[] = {"fdtd3d", "--3d", "--sizex", "64", "--same-size", "--use-pml", "--pml-type", "cpml",
                       "--cpml-kappa-max", "3.5", "--angle-teta", "30", "--output-dir", "/tmp/x", "--time-block", "5"};
    CHECK(s.parse(16, a) == fdtd::SETTINGS_OK);
    CHECK(s.sizeX == 64 && s.sizeY == 64 && s.sizeZ == 64);
    CHECK(s.doUsePML && s.pmlType == "cpml" && s.cpmlKappaMax == 3.5);
    CHECK(s.timeBlock == 5);
    CHECK(!s.help().empty() && !s.to_json().empty());
  }
  {
    fdtd::Settings s;
    const char* bad[] = {"fdtd3d", "--sizex", "not-a-number"};
    CHECK(s.parse(3, bad) != fdtd::SETTINGS_OK);
    const char* unk[] = {"fdtd3d", "--no-such-option"};
    fdtd::Settings s2;
    CHECK(s2.parse(2, unk) != fdtd::SETTINGS_OK);
    const char* missing[] = {"fdtd3d", "--sizex"};
    fdtd::Settings s3;
    CHECK(s3.parse(2, missing) != fdtd::SETTINGS_OK);
  }
  {
    fdtd::Settings s;
    std::vector<std::string> toks = {"--2d", "--sizex", "40", "--sizey", "30", "--dx", "0.001"};
    CHECK(s.parse(toks, false) == fdtd::SETTINGS_OK);
    CHECK(s.sizeX == 40 && s.sizeY == 30 && s.gridStep == 0.001);
  }
  for (int p : {1, 2, 3, 4, 6, 8, 12, 16}) {
    const fdtd::Int3 t = fdtd::optimal_topology({128, 96, 64}, p, {0, 1, 2});
    CHECK(t[0] * t[1] * t[2] == p);
    int covered = 0;
    for (int c = 0; c < t[0]; ++c) {
      int lo = 0, hi = 0;
      fdtd::chunk_bounds(128, t[0], c, lo, hi);
      CHECK(lo == covered && hi > lo);
      covered = hi;
    }
    CHECK(covered == 128);
  }
  CHECK(fdtd::halo_cost({64, 64, 64}, {2, 2, 2}) > 0.0);
  const std::string name = fdtd::grid_file_name(100, 3, "Ez", dir);
  CHECK(name.find("[100]") != std::string::npos && name.find("rank-3") != std::string::npos);
  std::vector<float> data(4096);
  for (size_t n = 0; n < data.size(); ++n) data[n] = 0.5f * (float)n;
  CHECK(fdtd::write_dat(dir + "/selftest.dat", data.data(), data.size() * sizeof(float)));
  std::vector<double> img(37 * 23);
  for (size_t n = 0; n < img.size(); ++n) img[n] = (double)((n * 7919) % 101) - 50.0;
  CHECK(fdtd::write_bmp(dir + "/selftest.bmp", img, 37, 23, "rgb"));
  CHECK(fdtd::write_bmp(dir + "/selftest-gray.bmp", img, 37, 23, "gray"));
  std::printf("host selftest: %d failed checks\n", g_fail);
  return g_fail ? 1 : 0;
}

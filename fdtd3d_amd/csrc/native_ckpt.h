// native_ckpt.h -- checkpoints of the native driver in the Python driver's format.
#pragma once
#include <hip/hip_runtime.h>

#include <functional>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "capi.h"
#include "settings_native.h"
#include "native_api.h"

// Part of the native driver: included by main.cpp only (one translation unit),
// hence the unnamed namespace.
namespace {

// ------------------------------------------------------------ checkpoints
// The Python driver's format (io/checkpoint.py): per state array a DAT file
// current[<step>]_rank-<r>_<name>.dat (raw values, z fastest) plus a JSON
// sidecar checkpoint[<step>]_rank-<r>.json.  The native driver writes and
// resumes the plain-media runs, whose state is the field components alone, so
// checkpoints move between the two drivers in both directions.
std::string ckpt_sidecar(const std::string& dir, long step) {
  return dir + "/checkpoint[" + std::to_string(step) + "]_rank-0.json";
}

// raw text of a top-level JSON value: a string's contents, a [...] list, or a scalar
std::string json_value(const std::string& j, const std::string& key, size_t from = 0) {
  const std::string k = "\"" + key + "\":";
  size_t p = j.find(k, from);
  if (p == std::string::npos) return "";
  p += k.size();
  while (p < j.size() && std::isspace((unsigned char)j[p])) ++p;
  if (p >= j.size()) return "";
  if (j[p] == '"') {
    const size_t e = j.find('"', p + 1);
    return e == std::string::npos ? "" : j.substr(p + 1, e - p - 1);
  }
  if (j[p] == '[') {
    const size_t e = j.find(']', p);
    return e == std::string::npos ? "" : j.substr(p, e - p + 1);
  }
  const size_t e = j.find_first_of(",}\n", p);
  std::string v = j.substr(p, e == std::string::npos ? std::string::npos : e - p);
  while (!v.empty() && std::isspace((unsigned char)v.back())) v.pop_back();
  return v;
}

std::vector<long> json_ints(const std::string& list) {
  std::vector<long> out;
  const char* c = list.c_str();
  while (*c) {
    if (*c == '-' || std::isdigit((unsigned char)*c)) {
      char* e = nullptr;
      out.push_back(std::strtol(c, &e, 10));
      c = e;
    } else {
      ++c;
    }
  }
  return out;
}

long ckpt_latest(const std::string& dir) {
  long best = -1;
  DIR* d = opendir(dir.c_str());
  if (!d) return -1;
  const std::string pre = "checkpoint[", suf = "]_rank-0.json";
  while (dirent* e = readdir(d)) {
    const std::string f = e->d_name;
    if (f.size() > pre.size() + suf.size() && f.compare(0, pre.size(), pre) == 0 &&
        f.compare(f.size() - suf.size(), suf.size(), suf) == 0)
      best = std::max(best, std::strtol(f.c_str() + pre.size(), nullptr, 10));
  }
  closedir(d);
  return best;
}

bool make_dirs(const std::string& dir) {
  for (size_t p = 1; p <= dir.size(); ++p)
    if (p == dir.size() || dir[p] == '/') {
      const std::string part = dir.substr(0, p);
      if (mkdir(part.c_str(), 0755) != 0 && errno != EEXIST) return false;
    }
  return true;
}

const char* const kCompNames[6] = {"Ex", "Ey", "Ez", "Hx", "Hy", "Hz"};

// Restores the present field components of a plain-media run; returns the
// checkpoint's step, or -1 (with a message) when the directory holds no
// matching checkpoint
// (`put(c, host)` places component c of the whole grid: the device array of a
// one-GPU run, every rank's allocated box of a --parallel-grid run)
template <typename T>
long ckpt_load(const fdtd::Settings& s, const std::string& scheme, const fdtd::Int3& N, const bool* present,
               const std::function<void(int, const std::vector<T>&)>& put) {
  const std::string& dir = s.loadFromFile;
  const long step = ckpt_latest(dir);
  if (step < 0) {
    std::fprintf(stderr, "fdtd3d: no checkpoint for rank 0 in %s\n", dir.c_str());
    return -1;
  }
  std::ifstream f(ckpt_sidecar(dir, step));
  std::stringstream buf;
  buf << f.rdbuf();
  const std::string j = buf.str();
  const std::vector<long> size = json_ints(json_value(j, "size")), shape = json_ints(json_value(j, "local_shape"));
  const std::vector<long> want = {N[0], N[1], N[2]};
  const char* bad = nullptr;
  if (json_value(j, "scheme") != scheme) bad = "scheme";
  else if (json_value(j, "dtype") != s.valueType) bad = "dtype";
  else if (json_value(j, "complex") != "false") bad = "complex";
  else if (size != want) bad = "size";
  else if (shape != want) bad = "local_shape";
  // a serial run's state: the whole grid at the origin, one rank, no
  // deep-halo sub-step in flight (the checks of io/checkpoint.py)
  else if (json_ints(json_value(j, "origin")) != std::vector<long>{0, 0, 0}) bad = "origin";
  else if (json_ints(json_value(j, "topology")) != std::vector<long>{1, 1, 1}) bad = "topology";
  else if (!json_value(j, "sub_step").empty() && json_value(j, "sub_step") != "0") bad = "sub_step";
  std::vector<std::string> names;
  for (size_t p = j.find("\"arrays\":"); p != std::string::npos;) {
    p = j.find("\"name\":", p);
    if (p == std::string::npos) break;
    names.push_back(json_value(j, "name", p));
    p += 7;
  }
  std::vector<std::string> fields;
  for (int c = 0; c < 6; ++c)
    if (present[c]) fields.push_back(kCompNames[c]);
  if (!bad && names != fields) bad = "arrays (a plain-media checkpoint holds the field components only)";
  if (bad) {
    std::fprintf(stderr, "fdtd3d: checkpoint %s mismatch in %s\n", bad, ckpt_sidecar(dir, step).c_str());
    return -1;
  }
  const size_t cells = (size_t)N[0] * N[1] * N[2];
  std::vector<T> host(cells);
  for (int c = 0; c < 6; ++c) {
    if (!present[c]) continue;
    const std::string path = fdtd::grid_file_name(step, 0, kCompNames[c], dir) + ".dat";
    std::ifstream in(path, std::ios::binary | std::ios::ate);
    if (!in || (size_t)in.tellg() != cells * sizeof(T)) {
      std::fprintf(stderr, "fdtd3d: %s missing or not %zu values\n", path.c_str(), cells);
      return -1;
    }
    in.seekg(0);
    in.read((char*)host.data(), (std::streamsize)(cells * sizeof(T)));
    put(c, host);
  }
  return step;
}

template <typename T>
long ckpt_load(const fdtd::Settings& s, const std::string& scheme, const fdtd::Int3& N, const bool* present,
               Dev<T>* F) {
  return ckpt_load<T>(s, scheme, N, present, [&](int c, const std::vector<T>& host) {
    HIP_OK(hipMemcpy(F[c].p, host.data(), host.size() * sizeof(T), hipMemcpyHostToDevice));
  });
}

// (`fetch(c, host)` fills component c of the whole grid; a --parallel-grid
// run gathers its ranks' owned blocks: the checkpoint is the serial form,
// which either driver resumes, decomposed or not)
template <typename T>
bool ckpt_save(const fdtd::Settings& s, const std::string& scheme, const fdtd::Int3& N, const bool* present,
               const std::function<void(int, std::vector<T>&)>& fetch, long step, double dx, double dt) {
  const std::string& dir = s.checkpointDir;
  if (!make_dirs(dir)) return false;
  const size_t cells = (size_t)N[0] * N[1] * N[2];
  std::vector<T> host(cells);
  char shape[96];
  std::snprintf(shape, sizeof(shape), "[%d, %d, %d]", N[0], N[1], N[2]);
  std::string arrays;
  for (int c = 0; c < 6; ++c) {
    if (!present[c]) continue;
    fetch(c, host);
    if (!fdtd::write_dat(fdtd::grid_file_name(step, 0, kCompNames[c], dir) + ".dat", host.data(), cells * sizeof(T)))
      return false;
    arrays += std::string(arrays.empty() ? "" : ", ") + "{\"name\": \"" + kCompNames[c] + "\", \"shape\": " + shape + "}";
  }
  std::ofstream f(ckpt_sidecar(dir, step));
  char num[64];
  f << "{\"format\": \"fdtd3d-amd-checkpoint-1\", \"version\": \"native\", \"step\": " << step
    << ", \"sub_step\": 0, \"scheme\": \"" << scheme << "\", \"size\": " << shape << ", \"dtype\": \""
    << s.valueType << "\", \"complex\": false, \"rank\": 0, \"topology\": [1, 1, 1], \"buffer_size\": 1"
    << ", \"lo\": [0, 0, 0], \"hi\": " << shape << ", \"origin\": [0, 0, 0], \"local_shape\": " << shape;
  std::snprintf(num, sizeof(num), "%.17g", dx);
  f << ", \"dx\": " << num;
  std::snprintf(num, sizeof(num), "%.17g", dt);
  f << ", \"dt\": " << num << ", \"arrays\": [" << arrays << "]}\n";
  return (bool)f;
}

template <typename T>
bool ckpt_save(const fdtd::Settings& s, const std::string& scheme, const fdtd::Int3& N, const bool* present,
               const Dev<T>* F, long step, double dx, double dt) {
  return ckpt_save<T>(s, scheme, N, present, [&](int c, std::vector<T>& host) {
    HIP_OK(hipMemcpy(host.data(), F[c].p, host.size() * sizeof(T), hipMemcpyDeviceToHost));
  }, step, dx, dt);
}

}  // namespace

// Native command-line parser generated from settings.inc.
#include "settings_native.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

namespace fdtd {

const char* solver_version() { return "0.3.0 (fdtd3d-amd, compatible with fdtd3d 0.2.2)"; }

namespace {

bool parse_int(const std::string& s, int& out) {
  char* end = nullptr;
  long v = std::strtol(s.c_str(), &end, 10);
  if (end == s.c_str() || *end != '\0') return false;
  out = (int)v;
  return true;
}

bool parse_double(const std::string& s, double& out) {
  char* end = nullptr;
  double v = std::strtod(s.c_str(), &end);
  if (end == s.c_str() || *end != '\0') return false;
  out = v;
  return true;
}

std::string json_escape(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    o += c;
  }
  return o;
}

}  // namespace

SettingsStatus Settings::parse(int argc, const char* const* argv, bool is_cmd, int first) {
  std::vector<std::string> tokens;
  for (int i = first; i < argc; ++i) tokens.emplace_back(argv[i]);
  return parse(tokens, is_cmd);
}

SettingsStatus Settings::parse(const std::vector<std::string>& t, bool is_cmd) {
  const size_t n = t.size();
  for (size_t i = 0; i < n; ++i) {
    const std::string& a = t[i];
    auto need_arg = [&](std::string& v) -> bool {
      if (i + 1 >= n) {
        message = "option " + a + " needs an argument";
        return false;
      }
      v = t[++i];
      return true;
    };
    std::string v;
    if (a == "--help") {
      message = help();
      return SETTINGS_BREAK;
    }
    if (a == "--version") {
      message = std::string("Version: ") + solver_version() + "\n";
      return SETTINGS_BREAK;
    }
#define FDTD_ACTION(cli, help)
#define FDTD_ACTION_ARG(cli, help)
#define FDTD_BOOL(field, cli, help) \
  if (a == cli) {                   \
    field = true;                   \
    continue;                       \
  }
#define FDTD_INT(field, cli, def, help)                         \
  if (a == cli) {                                               \
    if (!need_arg(v)) return SETTINGS_ERROR;                    \
    if (!parse_int(v, field)) {                                 \
      message = "option " + a + " expects an integer";          \
      return SETTINGS_ERROR;                                    \
    }                                                           \
    continue;                                                   \
  }
#define FDTD_FLOAT(field, cli, def, help)                       \
  if (a == cli) {                                               \
    if (!need_arg(v)) return SETTINGS_ERROR;                    \
    if (!parse_double(v, field)) {                              \
      message = "option " + a + " expects a number";            \
      return SETTINGS_ERROR;                                    \
    }                                                           \
    continue;                                                   \
  }
#define FDTD_STRING(field, cli, def, help)                      \
  if (a == cli) {                                               \
    if (!need_arg(v)) return SETTINGS_ERROR;                    \
    field = v;                                                  \
    continue;                                                   \
  }
#include "settings.inc"
#undef FDTD_ACTION
#undef FDTD_ACTION_ARG
#undef FDTD_BOOL
#undef FDTD_INT
#undef FDTD_FLOAT
#undef FDTD_STRING
    if (a == "--same-size") {
      sizeY = sizeZ = sizeX;
    } else if (a == "--same-size-pml") {
      pmlSizeY = pmlSizeZ = pmlSizeX;
    } else if (a == "--same-size-tfsf") {
      tfsfSizeY = tfsfSizeZ = tfsfSizeX;
    } else if (a == "--same-size-ntff") {
      ntffSizeY = ntffSizeZ = ntffSizeX;  // reference bug Settings.cpp:133-136 fixed
    } else if (a == "--same-size-topology") {
      topologySizeY = topologySizeZ = topologySizeX;
    } else if (a == "--1d") {
      dimension = 1;
    } else if (a == "--2d") {
      dimension = 2;
    } else if (a == "--3d") {
      dimension = 3;
    } else if (a == "--cmd-from-file") {
      if (!is_cmd) {
        message = "Command line files are not allowed in other command line files.\n";
        return SETTINGS_ERROR;
      }
      if (n != 2) {
        message = "Command line files are allowed only without other options.\n";
        return SETTINGS_ERROR;
      }
      if (!need_arg(v)) return SETTINGS_ERROR;
      std::ifstream in(v);
      if (!in) {
        message = "ERROR: Incorrect command line file.\n";
        return SETTINGS_ERROR;
      }
      std::vector<std::string> toks;
      std::string tok;
      while (in >> tok) toks.push_back(tok);  // (no fixed-size copies: reference bug Settings.cpp:249-250)
      return parse(toks, false);
    } else if (a == "--save-cmd-to-file") {
      if (!need_arg(v)) return SETTINGS_ERROR;
      std::ofstream out(v);
      for (size_t k = 0; k < n; ++k) {
        if (t[k] == "--save-cmd-to-file") {
          ++k;
          continue;
        }
        out << t[k] << "\n";
      }
    } else {
      message = "Unknown option [" + a + "]\n";
      return SETTINGS_UNKNOWN;
    }
  }
  return SETTINGS_OK;
}

SettingsStatus Settings::validate() {
  if (valueType != "f32" && valueType != "f64") {
    message = "--dtype must be f32 or f64";
    return SETTINGS_ERROR;
  }
  if (incidentWaveAngle1 < 0 || incidentWaveAngle1 > 90 || incidentWaveAngle2 < 0 || incidentWaveAngle2 > 90) {
    message = "--angle-teta and --angle-phi must be within [0, 90] degrees";
    return SETTINGS_ERROR;
  }
  if (bufferSize < 1 || sizeX < 1 || sizeY < 1 || sizeZ < 1) {
    message = "sizes and --buffer-size must be positive";
    return SETTINGS_ERROR;
  }
  return SETTINGS_OK;
}

std::string Settings::help() const {
  std::ostringstream o;
  char buf[64];
  o << "fdtd3d-amd: 1D, 2D and 3D FDTD electromagnetics solver for AMD Instinct MI355X "
       "(HIP kernels, RCCL domain decomposition).\n";
  o << "Usage: fdtd3d [options]\n\nOptions:\n";
#define FDTD_ACTION(cli, help) o << "  " << cli << "\n\t" << help << "\n";
#define FDTD_ACTION_ARG(cli, help) o << "  " << cli << " <string>\n\t" << help << "\n";
#define FDTD_BOOL(field, cli, help) o << "  " << cli << "\n\t" << help << "\n";
#define FDTD_INT(field, cli, def, help) o << "  " << cli << " <int> (default: " << def << ")\n\t" << help << "\n";
#define FDTD_FLOAT(field, cli, def, help)        \
  std::snprintf(buf, sizeof(buf), "%f", (double)def); \
  o << "  " << cli << " <float> (default: " << buf << ")\n\t" << help << "\n";
#define FDTD_STRING(field, cli, def, help) \
  o << "  " << cli << " <string> (default: " << def << ")\n\t" << help << "\n";
#include "settings.inc"
#undef FDTD_ACTION
#undef FDTD_ACTION_ARG
#undef FDTD_BOOL
#undef FDTD_INT
#undef FDTD_FLOAT
#undef FDTD_STRING
  o << "  --help\n\tPrint this help\n  --version\n\tPrint the version\n";
  return o.str();
}

std::string Settings::to_json() const {
  std::ostringstream o;
  o.precision(17);
  o << "{";
#define FDTD_ACTION(cli, help)
#define FDTD_ACTION_ARG(cli, help)
#define FDTD_BOOL(field, cli, help) o << "\"" #field "\": " << (field ? "true" : "false") << ", ";
#define FDTD_INT(field, cli, def, help) o << "\"" #field "\": " << field << ", ";
#define FDTD_FLOAT(field, cli, def, help) o << "\"" #field "\": " << field << ", ";
#define FDTD_STRING(field, cli, def, help) o << "\"" #field "\": \"" << json_escape(field) << "\", ";
#include "settings.inc"
#undef FDTD_ACTION
#undef FDTD_ACTION_ARG
#undef FDTD_BOOL
#undef FDTD_INT
#undef FDTD_FLOAT
#undef FDTD_STRING
  o << "\"dimension\": " << dimension << "}";
  return o.str();
}

}  // namespace fdtd

// C ABI for the Python parity test: parse argv, write the settings JSON.
extern "C" __attribute__((visibility("default"))) int fdtd_settings_parse_json(int argc, const char* const* argv,
                                                                                  char* out, int outlen) {
  fdtd::Settings s;
  int st = s.parse(argc, argv, true, 0);
  std::string j = (st == fdtd::SETTINGS_OK) ? s.to_json() : s.message;
  if ((int)j.size() + 1 > outlen) return -1;
  std::memcpy(out, j.c_str(), j.size() + 1);
  return st;
}

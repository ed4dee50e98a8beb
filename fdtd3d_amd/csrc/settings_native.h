// Native run-time settings (C++ side of fdtd3d_amd/utils/settings.py).
//
// Every field, default, flag name and help string is generated from
// settings.inc by X-macros, the same table the Python mirror parses, so the
// native driver and the Python driver accept exactly the same command lines
// (reference behaviour: Source/Settings/Settings.cpp:19-321).
#pragma once

#include <string>
#include <vector>

namespace fdtd {

enum SettingsStatus { SETTINGS_OK = 0, SETTINGS_ERROR = 1, SETTINGS_UNKNOWN = 2, SETTINGS_BREAK = 3 };

struct Settings {
#define FDTD_ACTION(cli, help)
#define FDTD_ACTION_ARG(cli, help)
#define FDTD_BOOL(field, cli, help) bool field = false;
#define FDTD_INT(field, cli, def, help) int field = def;
#define FDTD_FLOAT(field, cli, def, help) double field = def;
#define FDTD_STRING(field, cli, def, help) std::string field = def;
#include "settings.inc"
#undef FDTD_ACTION
#undef FDTD_ACTION_ARG
#undef FDTD_BOOL
#undef FDTD_INT
#undef FDTD_FLOAT
#undef FDTD_STRING

  int dimension = 3;
  std::string message;  // diagnostics of the last parse

  // Parse argv[first..argc); is_cmd = false when the tokens come from a file.
  SettingsStatus parse(int argc, const char* const* argv, bool is_cmd = true, int first = 1);
  SettingsStatus parse(const std::vector<std::string>& tokens, bool is_cmd);
  std::string help() const;
  std::string to_json() const;
  SettingsStatus validate();
};

const char* solver_version();

}  // namespace fdtd

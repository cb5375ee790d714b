// Host helpers that read hipBLASLt/Tensile kernel names (csrc/blas/lt_gemm.cpp; unit-tested under
// ASan/UBSan by csrc/tests/host_checks.cpp).
#pragma once

#include <cctype>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

namespace cs336 {

// Stream-K mode of a Tensile kernel name: the value of its "SK<n>" token (0 = data-parallel). Tokens
// that only start with SK (SKXCCM8, SKFTR0) are not it.
inline int stream_k_mode(const std::string& name) {
  size_t pos = 0;
  while ((pos = name.find("_SK", pos)) != std::string::npos) {
    size_t i = pos + 3, j = i;
    while (j < name.size() && std::isdigit(static_cast<unsigned char>(name[j]))) ++j;
    if (j > i && (j == name.size() || name[j] == '_')) return std::atoi(name.substr(i, j - i).c_str());
    pos = i;
  }
  return 0;
}

// Macro-tile area from a Tensile kernel name ("..._MT160x256x64_..." -> 160*256), 0 if absent.
inline int64_t macro_tile_area(const std::string& name) {
  const size_t pos = name.find("_MT");
  if (pos == std::string::npos) return 0;
  long a = 0, b = 0;
  if (std::sscanf(name.c_str() + pos + 3, "%ldx%ld", &a, &b) != 2) return 0;
  return int64_t(a) * int64_t(b);
}

}  // namespace cs336

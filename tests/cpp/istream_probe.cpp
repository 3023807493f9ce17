// istream_probe.cpp -- what `linestream >> a >> b >> c` (float) yields with this libstdc++, for the
// OBJ/MTL parser's edge cases (src/asset_utils/model_loader.cpp:59, 237).  One input line per
// case on stdin; prints "<ok> <bits a> <bits b> <bits c>" with the floats pre-set to a marker so
// untouched values show.  tests/test_producers.py pins oracle/scene_ref.py's restatement with it.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <sstream>
#include <string>

int main() {
  std::string line;
  while (std::getline(std::cin, line)) {
    std::istringstream ls(line);
    float v[3];
    const float marker = -12345.0f;
    v[0] = v[1] = v[2] = marker;
    const bool ok = static_cast<bool>(ls >> v[0] >> v[1] >> v[2]);
    uint32_t b[3];
    std::memcpy(b, v, sizeof b);
    std::printf("%d %08x %08x %08x\n", ok ? 1 : 0, b[0], b[1], b[2]);
  }
  return 0;
}

// Test harness (TEST INFRASTRUCTURE ONLY): runs yc_parse.h's json_check — the host build of the
// same function the gfx950 decoder runs — over "want hex" lines on stdin and reports mismatches.
#include <cstdio>
#include <vector>

#include "yc_parse.h"

int main() {
  int want;
  static char hex[1 << 16];
  int cases = 0, wrong = 0, refused = 0;
  while (scanf("%d %65535s", &want, hex) == 2) {
    std::vector<uint8_t> b;
    for (size_t i = 0; hex[i] && hex[i + 1]; i += 2) {
      unsigned v;
      sscanf(hex + i, "%2x", &v);
      b.push_back((uint8_t)v);
    }
    b.push_back(0);
    const uint32_t got = yc::json_check(b.data(), 0, (uint32_t)b.size() - 1);
    ++cases;
    if ((int)got == want) continue;
    if (want == 0 && got == yc::JSON_NONCANON) { ++refused; continue; }  // canonical, not verified: refused
    ++wrong;
    printf("want %d got %u: %s\n", want, got, hex);
  }
  printf("cases %d wrong %d refused %d\n", cases, wrong, refused);
  return wrong ? 1 : 0;
}

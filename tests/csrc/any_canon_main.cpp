// Test harness (TEST INFRASTRUCTURE ONLY): yc_parse.h any_content_canon — the host build of what
// the gfx950 rewrite kernel runs — over hex ContentAny contents (count + values) on stdin, one per
// line; prints the canonical content as hex, or "ERR <code>".
#include <cstdio>
#include <cstring>
#include <vector>

#include "yc_parse.h"

int main() {
  static char line[1 << 20];
  std::vector<uint32_t> arena(yc::JSON_ARENA_WORDS);
  while (fgets(line, sizeof line, stdin)) {
    std::vector<uint8_t> b;
    for (size_t i = 0; line[i] && line[i + 1] && line[i] != '\n'; i += 2) {
      unsigned v;
      sscanf(line + i, "%2x", &v);
      b.push_back((uint8_t)v);
    }
    const uint32_t n = (uint32_t)b.size();
    b.resize(n + 16, 0);
    uint32_t len = 0;
    const uint32_t r = yc::any_content_canon(b.data(), 0, n, nullptr, arena.data(), (uint32_t)arena.size(), len);
    if (r != yc::JSON_OK) { printf("ERR %u\n", r); continue; }
    std::vector<uint8_t> out(len + 1);
    uint32_t len2 = 0;
    yc::any_content_canon(b.data(), 0, n, out.data(), arena.data(), (uint32_t)arena.size(), len2);
    for (uint32_t i = 0; i < len2; ++i) printf("%02x", out[i]);
    printf("\n");
  }
}

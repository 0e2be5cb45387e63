// Test harness (TEST INFRASTRUCTURE ONLY): runs yc_parse.h's json_check and json_canon — the host
// build of the same functions the gfx950 decoder runs — over "want hex [canon-hex]" lines on stdin
// and reports mismatches: json_check's verdict (0 canonical, 1 JSON.parse throws, 2 otherwise; a
// canonical text it cannot judge may say 2, counted as "unjudged") and json_canon's text against
// Node's JSON.stringify(JSON.parse(s)).
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "yc_parse.h"

static std::vector<uint8_t> unhex(const char* hex) {
  std::vector<uint8_t> b;
  for (size_t i = 0; hex[i] && hex[i + 1]; i += 2) {
    unsigned v;
    sscanf(hex + i, "%2x", &v);
    b.push_back((uint8_t)v);
  }
  return b;
}

int main() {
  static char line[1 << 20];
  int cases = 0, wrong = 0, unjudged = 0, canon_wrong = 0, canon_checked = 0;
  std::vector<uint32_t> arena(1 << 16);
  while (fgets(line, sizeof line, stdin)) {
    int want = -1;
    char* sp = strchr(line, ' ');
    if (!sp) continue;
    want = atoi(line);
    char* hex = sp + 1;
    char* sp2 = strchr(hex, ' ');
    std::string chex;
    if (sp2) {
      *sp2 = 0;
      chex = sp2 + 1;
      while (!chex.empty() && (chex.back() == '\n' || chex.back() == '\r')) chex.pop_back();
    } else {
      size_t n = strlen(hex);
      while (n && (hex[n - 1] == '\n' || hex[n - 1] == '\r')) hex[--n] = 0;
    }
    std::vector<uint8_t> b = unhex(hex);
    const uint32_t n = (uint32_t)b.size();
    b.push_back(0);
    const uint32_t got = yc::json_check(b.data(), 0, n);
    ++cases;
    if ((int)got != want) {
      if (want == 0 && got == yc::JSON_NONCANON) ++unjudged;  // rewritten to itself below
      else { ++wrong; printf("check want %d got %u: %s\n", want, got, hex); }
    }
    uint32_t len = 0;
    const uint32_t r = yc::json_canon(b.data(), 0, n, nullptr, arena.data(), (uint32_t)arena.size(), len);
    if (want == 1) {
      if (r != yc::JSON_BAD) { ++canon_wrong; printf("canon accepts malformed (%u): %s\n", r, hex); }
      continue;
    }
    if (r != yc::JSON_OK) { ++canon_wrong; printf("canon refuses (%u): %s\n", r, hex); continue; }
    std::vector<uint8_t> out(len + 1);
    uint32_t len2 = 0;
    yc::json_canon(b.data(), 0, n, out.data(), arena.data(), (uint32_t)arena.size(), len2);
    out.resize(len2);
    const std::vector<uint8_t> want_c = want == 0 ? std::vector<uint8_t>(b.begin(), b.begin() + n) : unhex(chex.c_str());
    ++canon_checked;
    if (len2 != len || out != want_c) {
      ++canon_wrong;
      printf("canon differs: %s -> %.*s (want %.*s)\n", hex, (int)out.size(), (const char*)out.data(), (int)want_c.size(),
             (const char*)want_c.data());
    }
  }
  printf("cases %d wrong %d unjudged %d canon_checked %d canon_wrong %d\n", cases, wrong, unjudged, canon_checked, canon_wrong);
  return wrong || canon_wrong ? 1 : 0;
}

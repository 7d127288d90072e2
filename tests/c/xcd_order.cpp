// Host check of pqg::xcd_order (parquet-mr_amd/csrc/pqgpu_device.h): for every range size n and
// origin, a bijection of [0, n) in which the workgroups of each XCD take one contiguous run of
// indices in dispatch order. Built with hipcc (host code only) by tests/test_xcd_order.py.
#include <stdio.h>
#include <vector>

#include "pqgpu_device.h"

int main() {
  for (uint32_t n = 1; n <= 3000; n++) {
    for (uint32_t off = 0; off < 8; off++) {
      std::vector<int> seen(n, 0);
      std::vector<long> last(8, -1), lo(8, -1), hi(8, -1);
      for (uint32_t g = 0; g < n; g++) {
        const uint32_t p = pqg::xcd_order(g, n, off);
        if (p >= n || seen[p]++) { printf("FAIL n=%u off=%u g=%u p=%u\n", n, off, g, p); return 1; }
        const uint32_t x = (g + off) & 7u;
        if (last[x] >= 0 && (long)p != last[x] + 1) { printf("FAIL order n=%u off=%u g=%u\n", n, off, g); return 1; }
        last[x] = p;
      }
    }
  }
  printf("ok\n");
  return 0;
}

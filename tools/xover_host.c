/* xover_host.c -- the per-block host loop that a batched verify replaces, for
 * tools/crossover.py: CheckBlockIntegrity (hc_check_block, the library's host
 * path) over n uniform blocks, stopping at the first bad one, as the Go loops
 * of block_manager.go:203-235 and wal.go:366-403 do.  Measurement tooling, not
 * product code. */
#include <stdint.h>

#include "../include/hundcrc.h"

int64_t xo_check_loop(const uint8_t *base, uint64_t n, uint32_t bs) {
  for (uint64_t i = 0; i < n; i++)
    if (hc_check_block(base + i * (uint64_t)bs, bs) != HC_OK) return (int64_t)i;
  return -1;
}

/*
 * TEST INFRASTRUCTURE ONLY (the CPU baseline of the Zstd block compressor,
 * never the thing measured or shipped): port::Zstd_Compress
 * (port/port_stdcxx.h:133-161) driven per block exactly as TableBuilder::
 * WriteBlock drives it (table/table_builder.cc:172-185), timed on the host:
 *
 *   ZSTD_createCCtx; ZSTD_getCParams(level, max(n, 1), 0);
 *   ZSTD_CCtx_setCParams (1.5.x's definition: the seven ZSTD_CCtx_setParameter
 *   calls; libzstd 1.4.9 has no such function); ZSTD_compress2 into
 *   ZSTD_compressBound(n) bytes; ZSTD_freeCCtx.
 *
 *   zstd_port_bench BLOCKS_FILE BLOCK_BYTES LEVEL SECONDS PROCS
 *
 * Each of PROCS forked processes compresses the file's blocks round robin
 * (a distinct starting block each) for SECONDS; prints one JSON line with
 * the total rate in MB/s of uncompressed bytes and the output ratio.
 */
#define _POSIX_C_SOURCE 200809L
#define ZSTD_STATIC_LINKING_ONLY
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>
#include <zstd.h>

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static size_t port_compress(int level, const char* in, size_t n, char* out, size_t cap) {
  ZSTD_CCtx* ctx = ZSTD_createCCtx();
  ZSTD_compressionParameters p = ZSTD_getCParams(level, n > 1 ? n : 1, 0);
  ZSTD_CCtx_setParameter(ctx, ZSTD_c_windowLog, (int)p.windowLog);
  ZSTD_CCtx_setParameter(ctx, ZSTD_c_chainLog, (int)p.chainLog);
  ZSTD_CCtx_setParameter(ctx, ZSTD_c_hashLog, (int)p.hashLog);
  ZSTD_CCtx_setParameter(ctx, ZSTD_c_searchLog, (int)p.searchLog);
  ZSTD_CCtx_setParameter(ctx, ZSTD_c_minMatch, (int)p.minMatch);
  ZSTD_CCtx_setParameter(ctx, ZSTD_c_targetLength, (int)p.targetLength);
  ZSTD_CCtx_setParameter(ctx, ZSTD_c_strategy, (int)p.strategy);
  size_t r = ZSTD_compress2(ctx, out, cap, in, n);
  ZSTD_freeCCtx(ctx);
  return ZSTD_isError(r) ? 0 : r;
}

int main(int argc, char** argv) {
  if (argc != 6) {
    fprintf(stderr, "usage: %s BLOCKS_FILE BLOCK_BYTES LEVEL SECONDS PROCS\n", argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  fseek(f, 0, SEEK_END);
  const long total = ftell(f);
  fseek(f, 0, SEEK_SET);
  char* buf = malloc(total);
  if (fread(buf, 1, total, f) != (size_t)total) return 2;
  fclose(f);
  const size_t bs = strtoul(argv[2], 0, 10);
  const int level = atoi(argv[3]);
  const double secs = atof(argv[4]);
  const int procs = atoi(argv[5]);
  const size_t nb = total / bs;
  int fds[2];
  if (pipe(fds)) return 2;
  for (int pr = 0; pr < procs; ++pr) {
    if (fork() == 0) {
      const size_t cap = ZSTD_compressBound(bs);
      char* out = malloc(cap);
      double bytes = 0, outb = 0;
      size_t k = (size_t)pr * 7;
      const double t0 = now();
      double t = t0;
      while (t - t0 < secs) {
        for (int r = 0; r < 64; ++r, ++k) {
          outb += port_compress(level, buf + (k % nb) * bs, bs, out, cap);
          bytes += bs;
        }
        t = now();
      }
      double msg[3] = {bytes, outb, t - t0};
      if (write(fds[1], msg, sizeof msg) != sizeof msg) _exit(1);
      _exit(0);
    }
  }
  double bytes = 0, outb = 0, rate = 0;
  for (int pr = 0; pr < procs; ++pr) {
    double msg[3];
    if (read(fds[0], msg, sizeof msg) != sizeof msg) return 2;
    bytes += msg[0];
    outb += msg[1];
    rate += msg[0] / msg[2];
  }
  while (wait(NULL) > 0) {
  }
  printf("{\"procs\": %d, \"level\": %d, \"block_bytes\": %zu, \"MBps\": %.1f, \"output_pct\": %.2f, "
         "\"library\": \"%s\"}\n",
         procs, level, bs, rate / 1e6, 100.0 * outb / bytes, ZSTD_versionString());
  return 0;
}

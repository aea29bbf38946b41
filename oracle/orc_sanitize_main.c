/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see ekf_oracle.h). A standalone driver of the C oracle for
 * the host sanitizer build (`make -C oracle sanitize`: -fsanitize=address,undefined, the runtime
 * linked into this executable, so nothing is preloaded). tests/test_oracle_sanitize.py writes a
 * scenario the way orc.run_scenario drives the oracle — per message the wheel ticks through
 * DiffDrive::FKin (diff_drive.cpp:10-28), then fake_sensor_cb or sensor_cb (slam.cpp:180-316,
 * :318-530) — runs this binary and compares its output with the golden fixtures.
 *
 * Input (little-endian): int32 N, T, M, W, assoc, literal, joseph, pad; double track, radius;
 * per message: double wheel[W][2], int32 count, int32 ids[M], int32 actions[M], double rel[M][2].
 * Output: double poses[T][3], tmo[T][3]; int32 rcs[T], assoc_j[T][M], assoc_new[T][M];
 * double state[n], sigma[n][n], tmo[3]; uint32 counter.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ekf_oracle.h"

static void* xmalloc(size_t n) {
  void* p = calloc(1, n ? n : 1);
  if (!p) {
    fprintf(stderr, "out of memory\n");
    exit(2);
  }
  return p;
}

static void rd(void* p, size_t sz, size_t n, FILE* f) {
  if (fread(p, sz, n, f) != n) {
    fprintf(stderr, "short input\n");
    exit(2);
  }
}

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: %s <scenario.bin> <out.bin>\n", argv[0]);
    return 2;
  }
  FILE* in = fopen(argv[1], "rb");
  if (!in) return 2;
  int hdr[8];
  rd(hdr, sizeof(int), 8, in);
  const int N = hdr[0], T = hdr[1], M = hdr[2], W = hdr[3];
  const int assoc = hdr[4], literal = hdr[5], joseph = hdr[6];
  if (N < 1 || T < 0 || M < 0 || W < 0) return 2;
  double geo[2];
  rd(geo, sizeof(double), 2, in);
  const int n = 3 + 2 * N;
  orc_ekf* ekf = orc_ekf_create(N, 1e-2, 1e-2, 10e6, 2.0, literal);
  if (joseph) orc_ekf_set_joseph(ekf, 1);
  double dd[7] = {geo[0], geo[1], 0, 0, 0, 0, 0};
  double* poses = xmalloc(sizeof(double) * 3 * T);
  double* tmos = xmalloc(sizeof(double) * 3 * T);
  int* rcs = xmalloc(sizeof(int) * T);
  int* aj = xmalloc(sizeof(int) * T * M);
  int* an = xmalloc(sizeof(int) * T * M);
  double* wheel = xmalloc(sizeof(double) * 2 * W);
  int* ids = xmalloc(sizeof(int) * M);
  int* act = xmalloc(sizeof(int) * M);
  double* rel = xmalloc(sizeof(double) * 2 * M);
  double* x = xmalloc(sizeof(double) * n);
  for (int t = 0; t < T; ++t) {
    int c = 0;
    rd(wheel, sizeof(double), 2 * (size_t)W, in);
    rd(&c, sizeof(int), 1, in);
    rd(ids, sizeof(int), M, in);
    rd(act, sizeof(int), M, in);
    rd(rel, sizeof(double), 2 * (size_t)M, in);
    if (c < 0 || c > M) return 2;
    for (int k = 0; k < W; ++k) {
      double o[3];
      orc_fkin(dd, wheel[2 * k], wheel[2 * k + 1], o);
      orc_ekf_set_odom(ekf, o[0], o[1], o[2]);
    }
    for (int i = 0; i < M; ++i) aj[(size_t)t * M + i] = -1;
    if (assoc) {
      int* j = xmalloc(sizeof(int) * (c ? c : 1));
      int* nw = xmalloc(sizeof(int) * (c ? c : 1));
      rcs[t] = orc_ekf_sensor_cb(ekf, c, rel, j, nw);
      for (int i = 0; i < c; ++i) {
        aj[(size_t)t * M + i] = j[i];
        an[(size_t)t * M + i] = nw[i];
      }
      free(j);
      free(nw);
    } else {
      rcs[t] = orc_ekf_fake_sensor_cb(ekf, c, ids, act, rel);
    }
    unsigned cnt = 0;
    orc_ekf_get(ekf, x, NULL, tmos + 3 * t, &cnt);
    memcpy(poses + 3 * t, x, sizeof(double) * 3);
  }
  fclose(in);
  double* S = xmalloc(sizeof(double) * n * n);
  double tmo[3];
  unsigned counter = 0;
  orc_ekf_get(ekf, x, S, tmo, &counter);
  FILE* out = fopen(argv[2], "wb");
  if (!out) return 2;
  fwrite(poses, sizeof(double), 3 * (size_t)T, out);
  fwrite(tmos, sizeof(double), 3 * (size_t)T, out);
  fwrite(rcs, sizeof(int), T, out);
  fwrite(aj, sizeof(int), (size_t)T * M, out);
  fwrite(an, sizeof(int), (size_t)T * M, out);
  fwrite(x, sizeof(double), n, out);
  fwrite(S, sizeof(double), (size_t)n * n, out);
  fwrite(tmo, sizeof(double), 3, out);
  fwrite(&counter, sizeof(unsigned), 1, out);
  fclose(out);
  orc_ekf_destroy(ekf);
  free(poses);
  free(tmos);
  free(rcs);
  free(aj);
  free(an);
  free(wheel);
  free(ids);
  free(act);
  free(rel);
  free(x);
  free(S);
  return 0;
}

/*
 * wg_oracle_bench.c -- TEST INFRASTRUCTURE ONLY (see wg_oracle.h header comment).
 *
 * All-cores CPU baselines for bench.py's cpu_baseline legs: pthreads running
 * the oracle's restatement of the reference's Tun.Read / Tun.Write paths
 * (or_handle_virtio_read = tun/tun.go:514-632 + gro.go:1373-1493;
 * or_handle_gro = gro.go:1326-1367) on private copies of the same inputs.
 * Only the calls themselves are timed (per thread, CLOCK_MONOTONIC around each
 * call); restoring the inputs between calls is not, so the reported rate
 * (sum over threads of calls / call time) favours the CPU.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "wg_oracle.h"

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* ---- Tun.Read: handleVirtioRead over a set of super-packets ---- */
typedef struct {
  const uint8_t *arena;
  const size_t *offs, *lens;
  int n_jobs, first, nbufs, buf_len, offset;
  double seconds, busy;
  uint64_t calls;
} gso_arg;

static void *gso_worker(void *p) {
  gso_arg *a = (gso_arg *)p;
  size_t maxlen = 0;
  for (int j = 0; j < a->n_jobs; j++)
    if (a->lens[j] > maxlen) maxlen = a->lens[j];
  uint8_t *rb = malloc(maxlen + 16);
  uint8_t *mem = malloc((size_t)a->nbufs * a->buf_len);
  uint8_t **bufs = malloc(sizeof(uint8_t *) * a->nbufs);
  size_t *bl = malloc(sizeof(size_t) * a->nbufs);
  int *sizes = malloc(sizeof(int) * a->nbufs);
  for (int i = 0; i < a->nbufs; i++) {
    bufs[i] = mem + (size_t)i * a->buf_len;
    bl[i] = a->buf_len;
  }
  const double t_end = now_s() + a->seconds;
  int j = a->first % a->n_jobs;
  while (now_s() < t_end) {
    memcpy(rb, a->arena + a->offs[j], a->lens[j]); /* tun.file.Read into readBuf (not timed) */
    int n;
    const double t0 = now_s();
    or_handle_virtio_read(rb, a->lens[j], bufs, bl, a->nbufs, sizes, a->offset, &n);
    a->busy += now_s() - t0;
    a->calls++;
    j = (j + 1) % a->n_jobs;
  }
  free(rb); free(mem); free(bufs); free(bl); free(sizes);
  return NULL;
}

/* returns handleVirtioRead calls per second summed over `threads` threads */
double or_gso_bench_mt(const uint8_t *arena, const size_t *offs, const size_t *lens, int n_jobs, int nbufs,
                       int buf_len, int offset, int threads, double seconds, uint64_t *calls_out) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  gso_arg args[256];
  for (int t = 0; t < threads; t++) {
    args[t] = (gso_arg){arena, offs, lens, n_jobs, t * n_jobs / threads, nbufs, buf_len, offset, seconds, 0.0, 0};
    pthread_create(&th[t], NULL, gso_worker, &args[t]);
  }
  double rate = 0.0;
  uint64_t calls = 0;
  for (int t = 0; t < threads; t++) {
    pthread_join(th[t], NULL);
    if (args[t].busy > 0) rate += (double)args[t].calls / args[t].busy;
    calls += args[t].calls;
  }
  if (calls_out) *calls_out = calls;
  return rate;
}

/* ---- Tun.Write: handleGRO over one batch of packets (Go-slice buffers) ---- */
typedef struct {
  const uint8_t *pkts; /* packet k at pkts + k * stride, pkt_lens[k] bytes */
  const size_t *pkt_lens;
  size_t stride, cap;
  int n, offset, can_udp;
  double seconds, busy;
  uint64_t calls;
} gro_arg;

static void *gro_worker(void *p) {
  gro_arg *a = (gro_arg *)p;
  uint8_t *mem = calloc((size_t)a->n, a->cap);
  uint8_t **bufs = malloc(sizeof(uint8_t *) * a->n);
  size_t *lens = malloc(sizeof(size_t) * a->n), *caps = malloc(sizeof(size_t) * a->n);
  int *tw = malloc(sizeof(int) * a->n);
  const double t_end = now_s() + a->seconds;
  while (now_s() < t_end) {
    for (int i = 0; i < a->n; i++) { /* fresh Write batch (not timed) */
      bufs[i] = mem + (size_t)i * a->cap;
      memcpy(bufs[i] + a->offset, a->pkts + (size_t)i * a->stride, a->pkt_lens[i]);
      lens[i] = (size_t)a->offset + a->pkt_lens[i];
      caps[i] = a->cap;
    }
    int ntw;
    const double t0 = now_s();
    or_handle_gro(bufs, lens, caps, a->n, a->offset, a->can_udp, tw, &ntw);
    a->busy += now_s() - t0;
    a->calls++;
  }
  free(mem); free(bufs); free(lens); free(caps); free(tw);
  return NULL;
}

/* returns handleGRO calls per second summed over `threads` threads */
double or_gro_bench_mt(const uint8_t *pkts, const size_t *pkt_lens, size_t stride, int n, int offset, int can_udp,
                       int threads, double seconds, uint64_t *calls_out) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  gro_arg args[256];
  for (int t = 0; t < threads; t++) {
    args[t] = (gro_arg){pkts, pkt_lens, stride, 65535 + (size_t)offset, n, offset, can_udp, seconds, 0.0, 0};
    pthread_create(&th[t], NULL, gro_worker, &args[t]);
  }
  double rate = 0.0;
  uint64_t calls = 0;
  for (int t = 0; t < threads; t++) {
    pthread_join(th[t], NULL);
    if (args[t].busy > 0) rate += (double)args[t].calls / args[t].busy;
    calls += args[t].calls;
  }
  if (calls_out) *calls_out = calls;
  return rate;
}

/* ---- checksum batches: every thread runs whole passes over its own copy ---- */
typedef struct {
  int mode;
  const uint8_t *arena;
  size_t arena_len;
  const or_pkt *pkts;
  uint32_t n;
  double seconds, busy;
  uint64_t passes;
} cs_arg;

static void *cs_worker(void *p) {
  cs_arg *a = (cs_arg *)p;
  uint8_t *arena = malloc(a->arena_len + 64);
  uint8_t *out = malloc((size_t)a->n * 2 + 64);
  memcpy(arena, a->arena, a->arena_len);
  const double t_end = now_s() + a->seconds;
  while (now_s() < t_end) {
    const double t0 = now_s();
    or_checksum_batch(a->mode, arena, a->pkts, NULL, a->n, out, 0);
    a->busy += now_s() - t0;
    a->passes++;
  }
  free(arena);
  free(out);
  return NULL;
}

/* batch passes per second summed over `threads` threads (small batches: a
 * pass is too short to split one batch over threads) */
double or_checksum_bench_mt(int mode, const uint8_t *arena, size_t arena_len, const or_pkt *pkts, uint32_t n,
                            int threads, double seconds, uint64_t *passes_out) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  cs_arg args[256];
  for (int t = 0; t < threads; t++) {
    args[t] = (cs_arg){mode, arena, arena_len, pkts, n, seconds, 0.0, 0};
    pthread_create(&th[t], NULL, cs_worker, &args[t]);
  }
  double rate = 0.0;
  uint64_t passes = 0;
  for (int t = 0; t < threads; t++) {
    pthread_join(th[t], NULL);
    if (args[t].busy > 0) rate += (double)args[t].passes / args[t].busy;
    passes += args[t].passes;
  }
  if (passes_out) *passes_out = passes;
  return rate;
}

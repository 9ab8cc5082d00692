/*
 * split_hang_repro.c -- PROBE (not product): the round-5 teardown hang of
 * examples/rx_multigpu.c with a CU split (profiles/r05/README.md rows as/,
 * at/), replayed with the order that hung, step by step, every step stamped
 * on stderr, so that a run under the HIP runtime's own API log
 * (AMD_LOG_LEVEL=3) shows which call never returns and on which stream.
 *
 * The library now owns its split streams and refuses that order
 * (pptk_rx_stream_destroy -> -EBUSY), so this probe builds the two CU-masked
 * streams itself, as the round-5 library did, on an unsplit context:
 *   one-rank communicator, rounds of {batch on the rx stream with d_hash;
 *   event; the gather stream waits for it; pptk_rx_allgather_hash on the
 *   gather stream; event; the rx stream waits}, pptk_rx_comm_sync on both,
 *   then either
 *     order "old":  destroy the gather and rx streams, free the buffers,
 *                   destroy the context (its communicator) -- round 5's order
 *     order "new":  destroy the context first, then the streams.
 *
 *   gcc -O2 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude \
 *       tools/split_hang_repro.c -Lpptk_amd -lpptkrx -L/opt/rocm/lib -lamdhip64 -o repro
 *   timeout -k 5 60 ./repro old|new [rounds]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <hip/hip_runtime_api.h>


#include "pptk_rx.h"

static double t0;

static double now(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

#define STEP(what, call)                                                        \
  do {                                                                          \
    fprintf(stderr, "[%8.3f] >> %s\n", now() - t0, what);                       \
    long rc_ = (long)(call);                                                    \
    fprintf(stderr, "[%8.3f] << %s = %ld\n", now() - t0, what, rc_);            \
  } while (0)

int main(int argc, char **argv)
{
  const int old = argc > 1 && !strcmp(argv[1], "old");
  const int rounds = argc > 2 ? atoi(argv[2]) : 4;
  const uint64_t n = 1u << 16, stride = 1536;
  struct pptk_rx_opts o;
  struct pptk_rx_ctx *ctx = NULL;
  uint8_t uid[PPTK_RX_COMM_UID_BYTES];
  uint8_t *d_frames = NULL;
  struct pptk_rx_rec *d_recs = NULL;
  uint64_t *d_out = NULL;
  hipStream_t st = NULL, cs = NULL;
  hipEvent_t kdone, gdone;
  hipDeviceProp_t prop;
  uint32_t rxm[8] = {0}, csm[8] = {0};
  int ncu, i;

  setvbuf(stderr, NULL, _IONBF, 0);
  t0 = now();
  pptk_rx_opts_default(&o);
  o.comm_timeout_ms = 20000;
  STEP("pptk_rx_ctx_create", pptk_rx_ctx_create(&ctx, &o));
  STEP("pptk_rx_comm_uid", pptk_rx_comm_uid(uid));
  STEP("pptk_rx_comm_create(1, 0)", pptk_rx_comm_create(ctx, 1, 0, uid));
  STEP("hipGetDeviceProperties", hipGetDeviceProperties(&prop, 0));
  ncu = prop.multiProcessorCount;
  for (i = 0; i < ncu && i < 256; i++)
    (i >= ncu - 32 ? csm : rxm)[i / 32] |= 1u << (i % 32);
  STEP("hipExtStreamCreateWithCUMask(rx)", hipExtStreamCreateWithCUMask(&st, (uint32_t)((ncu + 31) / 32), rxm));
  STEP("hipExtStreamCreateWithCUMask(gather)", hipExtStreamCreateWithCUMask(&cs, (uint32_t)((ncu + 31) / 32), csm));
  STEP("hipEventCreate", hipEventCreateWithFlags(&kdone, hipEventDisableTiming));
  STEP("hipEventCreate", hipEventCreateWithFlags(&gdone, hipEventDisableTiming));
  STEP("hipMalloc frames", hipMalloc((void **)&d_frames, n * stride + 64));
  STEP("hipMalloc recs", hipMalloc((void **)&d_recs, n * 64));
  STEP("hipMalloc gather", hipMalloc((void **)&d_out, n * 8));
  STEP("hipMemset frames", hipMemset(d_frames, 0, n * stride + 64));
  for (i = 0; i < rounds; i++) {
    struct pptk_rx_dev_batch b;
    memset(&b, 0, sizeof(b));
    b.d_frames = d_frames;
    b.stride = stride;
    b.fixed_len = 1500;
    b.n = n;
    b.d_recs = d_recs;
    b.d_hash = d_out;
    STEP("pptk_rx_batch_device(rx stream)", pptk_rx_batch_device(ctx, &b, st));
    STEP("hipEventRecord(kdone, rx)", hipEventRecord(kdone, st));
    STEP("hipStreamWaitEvent(gather, kdone)", hipStreamWaitEvent(cs, kdone, 0));
    STEP("pptk_rx_allgather_hash(gather stream)", pptk_rx_allgather_hash(ctx, d_out, n, d_out, cs));
    STEP("hipEventRecord(gdone, gather)", hipEventRecord(gdone, cs));
    STEP("hipStreamWaitEvent(rx, gdone)", hipStreamWaitEvent(st, gdone, 0));
  }
  STEP("pptk_rx_comm_sync(gather)", pptk_rx_comm_sync(ctx, cs, 0));
  STEP("pptk_rx_comm_sync(rx)", pptk_rx_comm_sync(ctx, st, 0));
  STEP("hipEventDestroy", hipEventDestroy(kdone));
  STEP("hipEventDestroy", hipEventDestroy(gdone));
  if (old) {
    STEP("hipStreamDestroy(gather)", hipStreamDestroy(cs));
    STEP("hipStreamDestroy(rx)", hipStreamDestroy(st));
    STEP("hipFree frames", hipFree(d_frames));
    STEP("hipFree recs", hipFree(d_recs));
    STEP("hipFree gather", hipFree(d_out));
    STEP("hipDeviceSynchronize", hipDeviceSynchronize());
    fprintf(stderr, "[%8.3f] >> pptk_rx_ctx_destroy\n", now() - t0);
    pptk_rx_ctx_destroy(ctx);
    fprintf(stderr, "[%8.3f] << pptk_rx_ctx_destroy\n", now() - t0);
  } else {
    fprintf(stderr, "[%8.3f] >> pptk_rx_ctx_destroy\n", now() - t0);
    pptk_rx_ctx_destroy(ctx);
    fprintf(stderr, "[%8.3f] << pptk_rx_ctx_destroy\n", now() - t0);
    STEP("hipStreamDestroy(gather)", hipStreamDestroy(cs));
    STEP("hipStreamDestroy(rx)", hipStreamDestroy(st));
    STEP("hipFree frames", hipFree(d_frames));
    STEP("hipFree recs", hipFree(d_recs));
    STEP("hipFree gather", hipFree(d_out));
    STEP("hipDeviceSynchronize", hipDeviceSynchronize());
  }
  fprintf(stderr, "[%8.3f] done (%s order)\n", now() - t0, old ? "old" : "new");
  printf("split_hang_repro: %s order finished\n", old ? "old" : "new");
  return 0;
}

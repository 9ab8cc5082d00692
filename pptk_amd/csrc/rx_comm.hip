// rx_comm.hip -- multi-GPU part of the C-ABI (include/pptk_rx.h, "Multi-GPU").
//
// Packet batches shard embarrassingly: every GPU runs the
// receive transform on its own contiguous range of frames and the only
// exchange is one all-gather of the per-frame flow hashes, so that every
// GPU ends up with the flow hash of every frame of the batch.  That
// collective is RCCL's ncclAllGather over xGMI on a communicator owned by
// the context, enqueued on the caller's stream right behind the batch that
// produced the hashes (pptk_rx_dev_batch.d_hash), so it needs no host
// synchronisation and overlaps the next batch's kernel when the caller
// alternates streams.
//
// Two ways to build the communicator, matching the reference's two scaling
// models: one process per GPU (pptk_rx_comm_uid on one rank, the 128-byte id
// passed to every rank by the application, pptk_rx_comm_create on each), or
// one process driving every GPU with one rx thread per GPU, as LDP's
// multi-queue loops run one thread per queue (reference ldp/ldprecvmt.c:
// 174-182): pptk_rx_comm_create_all over one context per GPU.
//
// Errors: 0 or -errno; contract violations -EINVAL before RCCL is called,
// RCCL argument errors -EINVAL, every other RCCL or HIP failure -EIO.
#include <errno.h>
#include <string.h>

#include <new>
#include <vector>

#include <rccl/rccl.h>

#include "rx_internal.h"

using namespace pptk;

namespace {

struct RxComm {
  ncclComm_t comm = nullptr;
  int nranks = 0;
  int rank = 0;
};

int nccl_err(ncclResult_t r) {
  if (r == ncclSuccess) return 0;
  if (r == ncclInvalidArgument || r == ncclInvalidUsage) return -EINVAL;
  return -EIO;
}

RxComm *comm_of(const pptk_rx_ctx *c) { return (RxComm *)*ctx_comm_slot((pptk_rx_ctx *)c); }

}  // namespace

namespace pptk {

void comm_release(pptk_rx_ctx *c) {
  RxComm *m = comm_of(c);
  if (!m) return;
  (void)ncclCommDestroy(m->comm);
  delete m;
  *ctx_comm_slot(c) = nullptr;
}

}  // namespace pptk

extern "C" {

int pptk_rx_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return -EIO;
  return n;
}

int pptk_rx_comm_uid(uint8_t uid[PPTK_RX_COMM_UID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) == PPTK_RX_COMM_UID_BYTES, "RCCL unique id size");
  if (!uid) return -EINVAL;
  ncclUniqueId id;
  const int rc = nccl_err(ncclGetUniqueId(&id));
  if (rc == 0) memcpy(uid, &id, sizeof(id));
  return rc;
}

int pptk_rx_comm_create(struct pptk_rx_ctx *c, int nranks, int rank,
                        const uint8_t uid[PPTK_RX_COMM_UID_BYTES]) {
  if (!c || !uid || nranks < 1 || rank < 0 || rank >= nranks) return -EINVAL;
  if (comm_of(c)) return -EINVAL;   // one communicator per context
  RxComm *m = new (std::nothrow) RxComm();
  if (!m) return -ENOMEM;
  ncclUniqueId id;
  memcpy(&id, uid, sizeof(id));
  int rc;
  {
    DeviceScope ds(ctx_device(c));
    rc = ds.ok ? nccl_err(ncclCommInitRank(&m->comm, nranks, id, rank)) : -EIO;
  }
  if (rc != 0) {
    delete m;
    return rc;
  }
  m->nranks = nranks;
  m->rank = rank;
  *ctx_comm_slot(c) = m;
  return 0;
}

int pptk_rx_comm_create_all(struct pptk_rx_ctx *const *ctxs, int n) {
  if (!ctxs || n < 1) return -EINVAL;
  std::vector<int> devs((size_t)n);
  for (int i = 0; i < n; ++i) {
    if (!ctxs[i] || comm_of(ctxs[i])) return -EINVAL;
    devs[(size_t)i] = ctx_device(ctxs[i]);
    for (int k = 0; k < i; ++k)   // one rank per GPU
      if (devs[(size_t)k] == devs[(size_t)i] || ctxs[k] == ctxs[i]) return -EINVAL;
  }
  std::vector<ncclComm_t> comms((size_t)n, nullptr);
  int rc;
  {
    DeviceScope ds(devs[0]);   // (ncclCommInitAll sets each device itself)
    rc = nccl_err(ncclCommInitAll(comms.data(), n, devs.data()));
  }
  if (rc != 0) return rc;
  for (int i = 0; i < n; ++i) {
    RxComm *m = new (std::nothrow) RxComm();
    if (!m) {
      for (int k = 0; k < n; ++k) {
        if (k < i) comm_release(ctxs[k]);
        else (void)ncclCommDestroy(comms[(size_t)k]);
      }
      return -ENOMEM;
    }
    m->comm = comms[(size_t)i];
    m->nranks = n;
    m->rank = i;
    *ctx_comm_slot(ctxs[i]) = m;
  }
  return 0;
}

int pptk_rx_comm_destroy(struct pptk_rx_ctx *c) {
  if (!c) return -EINVAL;
  DeviceScope ds(ctx_device(c));
  comm_release(c);
  return 0;
}

int pptk_rx_comm_info(const struct pptk_rx_ctx *c, int *nranks, int *rank) {
  if (!c) return -EINVAL;
  const RxComm *m = comm_of(c);
  if (!m) return -EINVAL;
  if (nranks) *nranks = m->nranks;
  if (rank) *rank = m->rank;
  return 0;
}

void pptk_rx_shard_range(uint64_t n, int nranks, int rank, uint64_t *first, uint64_t *count,
                         uint64_t *per_rank) {
  uint64_t per = 0, lo = 0, cnt = 0;
  if (nranks >= 1 && rank >= 0 && rank < nranks) {
    per = (n + (uint64_t)nranks - 1) / (uint64_t)nranks;
    lo = (uint64_t)rank * per;
    if (lo > n) lo = n;
    cnt = n - lo < per ? n - lo : per;
  }
  if (first) *first = lo;
  if (count) *count = cnt;
  if (per_rank) *per_rank = per;
}

int pptk_rx_allgather_hash(struct pptk_rx_ctx *c, const uint64_t *d_hash, uint64_t n,
                           uint64_t *d_out, void *stream) {
  if (!c) return -EINVAL;
  RxComm *m = comm_of(c);
  if (!m) return -EINVAL;
  if (n == 0) return 0;
  if (!d_hash || !d_out) return -EINVAL;
  DeviceScope ds(ctx_device(c));
  if (!ds.ok) return -EIO;
  return nccl_err(ncclAllGather(d_hash, d_out, (size_t)n, ncclUint64, m->comm,
                                (hipStream_t)stream));
}

}  // extern "C"

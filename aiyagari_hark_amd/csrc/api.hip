// Handle lifecycle, errors and the RCCL binding of libaiyagari.
#include "internal.h"

#include <cstring>
#include <new>

extern "C" int32_t aiy_version(void) { return 210; }  // 0.2.1: Krusell-Smith employment

extern "C" int32_t aiy_create(int32_t device, aiy_handle** out) {
  if (!out) return AIY_ERR_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return AIY_ERR_HIP;
  if (device < 0 || device >= n) return AIY_ERR_ARG;
  aiy_handle* h = new (std::nothrow) aiy_handle();
  if (!h) return AIY_ERR_STATE;
  h->device = device;
  if (hipSetDevice(device) != hipSuccess) {
    delete h;
    return AIY_ERR_HIP;
  }
  *out = h;
  return AIY_OK;
}

extern "C" int32_t aiy_destroy(aiy_handle* h) {
  if (!h) return AIY_OK;
  (void)hipSetDevice(h->device);
  if (h->comm && h->comm_owned) (void)ncclCommDestroy(h->comm);
  if (h->d_dist) (void)hipFree(h->d_dist);
  if (h->d_last) (void)hipFree(h->d_last);
  if (h->d_egm_hint) (void)hipFree(h->d_egm_hint);
  if (h->d_egm_aa) (void)hipFree(h->d_egm_aa);
  if (h->h_dist) (void)hipHostFree(h->h_dist);
  if (h->h_last) (void)hipHostFree(h->h_last);
  if (h->d_partials) (void)hipFree(h->d_partials);
  if (h->d_ticket) (void)hipFree(h->d_ticket);
  if (h->cap_stream) (void)hipStreamDestroy(h->cap_stream);
  if (h->d_blk) (void)hipFree(h->d_blk);
  if (h->d_res_sync) (void)hipFree(h->d_res_sync);
  for (hipEvent_t e : h->res_ev)
    if (e) (void)hipEventDestroy(e);
  if (h->h_blk) (void)hipHostFree(h->h_blk);
  if (h->d_hdist) (void)hipFree(h->d_hdist);
  if (h->d_K) (void)hipFree(h->d_K);
  if (h->d_hlast) (void)hipFree(h->d_hlast);
  if (h->d_stats) (void)hipFree(h->d_stats);
  if (h->h_hdist) (void)hipHostFree(h->h_hdist);
  if (h->h_K) (void)hipHostFree(h->h_K);
  if (h->h_hlast) (void)hipHostFree(h->h_hlast);
  if (h->hand_ev) (void)hipEventDestroy(h->hand_ev);
  if (h->d_ge) (void)hipFree(h->d_ge);
  for (hipEvent_t e : h->ge_ev)
    if (e) (void)hipEventDestroy(e);
  if (h->d_hc) (void)hipFree(h->d_hc);
  if (h->d_hcd) (void)hipFree(h->d_hcd);
  for (hipEvent_t e : h->hc_ev)
    if (e) (void)hipEventDestroy(e);
  delete h;
  return AIY_OK;
}

extern "C" const char* aiy_last_error(const aiy_handle* h) { return h ? h->err.c_str() : "null handle"; }

extern "C" int32_t aiy_comm_unique_id(void* out128) {
  if (!out128) return AIY_ERR_ARG;
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId must be 128 bytes");
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return AIY_ERR_COMM;
  std::memcpy(out128, &id, sizeof(id));
  return AIY_OK;
}

extern "C" int32_t aiy_comm_init(aiy_handle* h, const void* unique_id128, int32_t nranks, int32_t rank) {
  if (!h) return AIY_ERR_ARG;
  if (!unique_id128 || nranks < 1 || rank < 0 || rank >= nranks) return aiy::fail(h, AIY_ERR_ARG, "bad comm args");
  if (h->comm) return aiy::fail(h, AIY_ERR_STATE, "communicator already bound");
  AIY_HIP(h, hipSetDevice(h->device));
  ncclUniqueId id;
  std::memcpy(&id, unique_id128, sizeof(id));
  ncclResult_t r = ncclCommInitRank(&h->comm, nranks, id, rank);
  if (r != ncclSuccess) {
    h->comm = nullptr;
    return aiy::fail(h, AIY_ERR_COMM, "ncclCommInitRank: %s", ncclGetErrorString(r));
  }
  h->nranks = nranks;
  h->rank = rank;
  h->comm_owned = true;
  return AIY_OK;
}

// Borrow a communicator the caller owns (e.g. torch.distributed's RCCL process group, whose
// ncclComm_t ProcessGroupNCCL._comm_ptr() returns): the library enqueues its all-reduces on
// it and never destroys it, so a process keeps ONE communicator per device.  The caller keeps
// it alive until aiy_comm_destroy (which only unbinds it) or aiy_destroy.
extern "C" int32_t aiy_comm_bind(aiy_handle* h, void* comm) {
  if (!h) return AIY_ERR_ARG;
  if (!comm) return aiy::fail(h, AIY_ERR_ARG, "null communicator");
  if (h->comm) return aiy::fail(h, AIY_ERR_STATE, "communicator already bound");
  ncclComm_t c = static_cast<ncclComm_t>(comm);
  int nranks = 0, rank = 0, dev = -1;
  ncclResult_t r = ncclCommCount(c, &nranks);
  if (r == ncclSuccess) r = ncclCommUserRank(c, &rank);
  if (r == ncclSuccess) r = ncclCommCuDevice(c, &dev);
  if (r != ncclSuccess) return aiy::fail(h, AIY_ERR_COMM, "communicator query: %s", ncclGetErrorString(r));
  if (dev != h->device) return aiy::fail(h, AIY_ERR_ARG, "communicator is on device %d, handle on %d", dev, h->device);
  h->comm = c;
  h->comm_owned = false;
  h->nranks = nranks;
  h->rank = rank;
  return AIY_OK;
}

extern "C" int32_t aiy_comm_destroy(aiy_handle* h) {
  if (!h) return AIY_ERR_ARG;
  if (h->comm && h->comm_owned) (void)ncclCommDestroy(h->comm);
  h->comm = nullptr;
  h->comm_owned = false;
  h->nranks = 1;
  h->rank = 0;
  return AIY_OK;
}

extern "C" int32_t aiy_allreduce_sum(aiy_handle* h, double* buf, int64_t n, aiy_stream stream) {
  if (!h) return AIY_ERR_ARG;
  if (!h->comm) return aiy::fail(h, AIY_ERR_STATE, "no communicator bound");
  if (!buf || n < 0) return aiy::fail(h, AIY_ERR_ARG, "bad buffer");
  ncclResult_t r = ncclAllReduce(buf, buf, (size_t)n, ncclDouble, ncclSum, h->comm, aiy::as_stream(stream));
  if (r != ncclSuccess) return aiy::fail(h, AIY_ERR_COMM, "ncclAllReduce: %s", ncclGetErrorString(r));
  return AIY_OK;
}

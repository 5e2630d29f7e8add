// comm.hip — the Lloyd step's all-reduce issued from C: an RCCL communicator
// owned by the context (one process per GPU, RCCL over xGMI), so that a whole
// step — assign, SUM all-reduce of the k x (d+1) int64 sums, finalize — is
// enqueued by one call with no Python between the kernels and the collective
// (the reference is single-process: src/kmeans_plusplus.py:31-48; SURVEY §5
// "a single fused all-reduce per step").
//
// librccl is bound at run time (dlopen + dlsym): a process that already loaded
// torch's librccl.so (soname librccl.so.1) shares that copy; otherwise ROCm's.
// Nothing links against it, so a host without RCCL still loads libcdr and
// only cdr_comm_* report CDR_ERR_UNSUPPORTED.
#include <dlfcn.h>
#include <link.h>

#include <cstring>
#include <mutex>

#include <rccl/rccl.h>

#include "cdr_internal.h"

namespace cdr {

namespace {

struct Rccl {
  bool tried = false, ok = false;
  std::string why;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};

Rccl g_rccl;
std::mutex g_rccl_mu;

// path of an already-loaded librccl (torch's), if any
int find_loaded(struct dl_phdr_info* info, size_t, void* out) {
  const char* p = info->dlpi_name;
  if (p && std::strstr(p, "librccl.so")) {
    *static_cast<std::string*>(out) = p;
    return 1;
  }
  return 0;
}

Rccl& rccl() {
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  Rccl& r = g_rccl;
  if (r.tried) return r;
  r.tried = true;
  std::string loaded;
  dl_iterate_phdr(find_loaded, &loaded);
  void* h = nullptr;
  const char* cands[] = {loaded.empty() ? nullptr : loaded.c_str(), "librccl.so.1",
                         "/opt/rocm/lib/librccl.so.1"};
  for (const char* c : cands) {
    if (!c) continue;
    h = dlopen(c, RTLD_NOW | RTLD_LOCAL);
    if (h) break;
  }
  if (!h) {
    r.why = "librccl not found";
    return r;
  }
  r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
  r.init_rank = reinterpret_cast<decltype(r.init_rank)>(dlsym(h, "ncclCommInitRank"));
  r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(h, "ncclAllReduce"));
  r.all_gather = reinterpret_cast<decltype(r.all_gather)>(dlsym(h, "ncclAllGather"));
  r.destroy = reinterpret_cast<decltype(r.destroy)>(dlsym(h, "ncclCommDestroy"));
  r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
  r.ok = r.get_unique_id && r.init_rank && r.all_reduce && r.all_gather && r.destroy &&
         r.error_string;
  if (!r.ok) r.why = "librccl lacks ncclGetUniqueId / ncclCommInitRank / ncclAllReduce / ncclAllGather";
  return r;
}

Rccl& need_rccl() {
  Rccl& r = rccl();
  if (!r.ok) CDR_FAIL(CDR_ERR_UNSUPPORTED, "RCCL unavailable: " + r.why);
  return r;
}

void nccl_check(ncclResult_t e, const char* what) {
  if (e != ncclSuccess)
    CDR_FAIL(CDR_ERR_HIP, std::string(what) + " failed: " + g_rccl.error_string(e));
}

}  // namespace

// SUM all-reduce of n int64 in place on the context stream (the step's sums).
void comm_allreduce_i64(Ctx& c, long long* buf, size_t n) {
  Rccl& r = need_rccl();
  nccl_check(r.all_reduce(buf, buf, n, ncclInt64, ncclSum, static_cast<ncclComm_t>(c.comm),
                          c.stream),
             "ncclAllReduce");
}

// SUM all-reduce of n doubles in place (seeding: the picked row, its index
// and the flags; every other rank contributes zeros, so the sum is exact).
void comm_allreduce_f64(Ctx& c, double* buf, size_t n) {
  Rccl& r = need_rccl();
  if (!c.comm) CDR_FAIL(CDR_ERR_STATE, "no communicator (cdr_comm_init)");
  nccl_check(r.all_reduce(buf, buf, n, ncclFloat64, ncclSum, static_cast<ncclComm_t>(c.comm),
                          c.stream),
             "ncclAllReduce");
}

// In-place all-gather: `bytes` per rank, this rank's part at buf + rank * bytes.
void comm_allgather(Ctx& c, void* buf, size_t bytes) {
  Rccl& r = need_rccl();
  if (!c.comm) CDR_FAIL(CDR_ERR_STATE, "no communicator (cdr_comm_init)");
  unsigned char* b = static_cast<unsigned char*>(buf);
  nccl_check(r.all_gather(b + (size_t)c.comm_rank * bytes, b, bytes, ncclUint8,
                          static_cast<ncclComm_t>(c.comm), c.stream),
             "ncclAllGather");
}

void comm_release(Ctx& c) {
  if (c.comm && g_rccl.ok) (void)g_rccl.destroy(static_cast<ncclComm_t>(c.comm));
  c.comm = nullptr;
  c.comm_ranks = 1;
  c.comm_rank = 0;
}

}  // namespace cdr

using namespace cdr;

extern "C" {

int cdr_comm_available(int32_t* ok) {
  CDR_TRY
  if (!ok) CDR_FAIL(CDR_ERR_ARG, "null argument");
  *ok = rccl().ok ? 1 : 0;  // dlopen + dlsym only: no bootstrap listener
  CDR_CATCH
}

int cdr_comm_ranks(cdr_ctx* h, int32_t* nranks, int32_t* rank) {
  CDR_TRY
  if (!h || !nranks || !rank) CDR_FAIL(CDR_ERR_ARG, "null argument");
  *nranks = h->c.comm ? h->c.comm_ranks : 0;  // 0: no communicator
  *rank = h->c.comm ? h->c.comm_rank : 0;
  CDR_CATCH
}

int cdr_comm_unique_id(void* id128) {
  CDR_TRY
  if (!id128) CDR_FAIL(CDR_ERR_ARG, "null argument");
  Rccl& r = need_rccl();
  ncclUniqueId id;
  nccl_check(r.get_unique_id(&id), "ncclGetUniqueId");
  static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
  std::memcpy(id128, &id, sizeof(id));
  CDR_CATCH
}

int cdr_comm_init(cdr_ctx* h, const void* id128, int32_t nranks, int32_t rank) {
  CDR_TRY
  if (!h || !id128) CDR_FAIL(CDR_ERR_ARG, "null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) CDR_FAIL(CDR_ERR_ARG, "bad rank / nranks");
  Ctx& c = h->c;
  HIP_CHECK(hipSetDevice(c.device));
  Rccl& r = need_rccl();
  comm_release(c);
  ncclUniqueId id;
  std::memcpy(&id, id128, sizeof(id));
  ncclComm_t comm = nullptr;
  nccl_check(r.init_rank(&comm, nranks, id, rank), "ncclCommInitRank");
  c.comm = comm;
  c.comm_ranks = nranks;
  c.comm_rank = rank;
  CDR_CATCH
}

int cdr_comm_destroy(cdr_ctx* h) {
  CDR_TRY
  if (!h) CDR_FAIL(CDR_ERR_ARG, "null ctx");
  HIP_CHECK(hipSetDevice(h->c.device));
  HIP_CHECK(hipStreamSynchronize(h->c.stream));
  comm_release(h->c);
  CDR_CATCH
}

}  // extern "C"

// bg_group.hip — multi-GPU: chromosome shards on several devices, reassembled over RCCL.
//
// The reference scales out per chromosome (docs/content/reference/set-operations/
// bedops.rst:721-726): every comparator starts with strcmp(chrom) (BedCompare.hpp:42-43,
// BedDistances.hpp:59-60,99-100), so whole chromosomes are independent. A group is one
// bg_ctx per device: each member loads and processes only the chromosomes assigned to
// it (the caller assigns them; host text goes to each GPU over its own link), formats
// its output in HBM, and bg_group_gather reassembles the per-chromosome texts on member
// 0 in the global (strcmp) chromosome order with one grouped round of ncclSend/ncclRecv
// over xGMI — the path's only exchange. Two shapes:
//   bg_group_open       one process driving n devices (ncclCommInitAll): the C front-ends
//                       under BEDGPU_DEVICES=0,1,...
//   bg_group_open_rank  one rank per process (ncclCommInitRank from a unique id that the
//                       caller distributes): bench.py under torch.distributed.run
// A device listed twice (tests on a one-GPU machine) gets no communicator; transfers then
// are device-local copies and the sizes are exchanged on the host.
#include <dlfcn.h>
#include <rccl/rccl.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "bg_internal.h"

// RCCL is loaded on first use (dlopen), not linked: librccl is a 570 MB library whose load
// and fat-binary registration would otherwise be paid by every single-GPU run of the CLIs at
// process start. The header gives the types; these pointers are the entry points.
namespace {
struct Rccl {
  bool ok = false;
  std::string err;
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitAll) CommInitAll = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclAllReduce) AllReduce = nullptr;
  decltype(&ncclSend) Send = nullptr;
  decltype(&ncclRecv) Recv = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
};
Rccl& rccl() {
  static Rccl R;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* e = dlerror();
      R.err = e ? e : "dlopen librccl.so.1 failed";
      return;
    }
#define BG_SYM(f)                                                         \
  R.f = reinterpret_cast<decltype(R.f)>(dlsym(h, "nccl" #f));             \
  if (!R.f) {                                                             \
    R.err = "librccl.so.1 lacks nccl" #f;                                 \
    return;                                                               \
  }
    BG_SYM(GetUniqueId) BG_SYM(CommInitAll) BG_SYM(CommInitRank) BG_SYM(CommDestroy) BG_SYM(AllReduce)
    BG_SYM(Send) BG_SYM(Recv) BG_SYM(GroupStart) BG_SYM(GroupEnd) BG_SYM(GetErrorString)
#undef BG_SYM
    R.ok = true;
  });
  return R;
}
}  // namespace
#define ncclGetUniqueId rccl().GetUniqueId
#define ncclCommInitAll rccl().CommInitAll
#define ncclCommInitRank rccl().CommInitRank
#define ncclCommDestroy rccl().CommDestroy
#define ncclAllReduce rccl().AllReduce
#define ncclSend rccl().Send
#define ncclRecv rccl().Recv
#define ncclGroupStart rccl().GroupStart
#define ncclGroupEnd rccl().GroupEnd
#define ncclGetErrorString rccl().GetErrorString

struct bg_group {
  std::vector<bg_ctx*> ctx;      // local members
  std::vector<ncclComm_t> comm;  // one per local member (empty: no RCCL, single process)
  int nranks = 1;                // global members
  int rank0 = 0;                 // global index of local member 0
  // BEDGPU_RCCL_SELF=1 on a one-member group: a one-rank communicator, and member 0's own
  // runs go through ncclSend/ncclRecv to itself instead of device copies, so the
  // communicator branch of bg_group_gather (all-reduce of the sizes, grouped send/recv,
  // group error paths) runs on a one-GPU machine (tests/test_gpu_shard.py)
  bool self = false;
};

// a group that cannot be opened has no context to keep the message in: say why on stderr
static void group_warn(const std::string& m) { fprintf(stderr, "bedgpu: group: %s\n", m.c_str()); }
static void group_warn_nccl(ncclResult_t r, const char* what) {
  group_warn(std::string(what) + ": " + (ncclGetErrorString ? ncclGetErrorString(r) : "RCCL error"));
}

static int nccl_fail(bg_ctx* c, ncclResult_t r, const char* what) {
  return bg_fail(c, BG_E_HIP, std::string("RCCL error: ") + ncclGetErrorString(r) + " in " + what);
}
#define BG_NCCL(c, expr)                                   \
  do {                                                     \
    ncclResult_t _r = (expr);                              \
    if (_r != ncclSuccess) return nccl_fail((c), _r, #expr); \
  } while (0)

extern "C" int bg_group_uid(void* uid) {
  if (!uid) return BG_E_ARG;
  if (!rccl().ok) return BG_E_HIP;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return BG_E_HIP;
  static_assert(sizeof(ncclUniqueId) <= BG_UID_BYTES, "unique id size");
  memset(uid, 0, BG_UID_BYTES);
  memcpy(uid, &id, sizeof(id));
  return 0;
}

extern "C" int bg_group_open(bg_group** out, const int* devices, int n) {
  if (!out || !devices || n < 1) return BG_E_ARG;
  *out = nullptr;
  bg_group* g = new bg_group();
  bool distinct = true;
  for (int i = 0; i < n; ++i) {
    for (int j = 0; j < i; ++j) distinct = distinct && devices[j] != devices[i];
    bg_ctx* c = nullptr;
    int rc = bg_open(&c, devices[i]);
    if (rc) {
      bg_group_close(g);
      return rc;
    }
    g->ctx.push_back(c);
  }
  g->nranks = n;
  const char* se = getenv("BEDGPU_RCCL_SELF");
  g->self = n == 1 && se && strcmp(se, "0") != 0;
  if ((distinct && n > 1) || g->self) {
    if (!rccl().ok) {
      bg_fail(g->ctx[0], BG_E_HIP, "RCCL unavailable: " + rccl().err);
      group_warn("RCCL unavailable: " + rccl().err);
      bg_group_close(g);
      return BG_E_HIP;
    }
    g->comm.resize(n);
    const ncclResult_t ri = ncclCommInitAll(g->comm.data(), n, devices);
    if (ri != ncclSuccess) {
      group_warn_nccl(ri, "ncclCommInitAll");
      g->comm.clear();
      bg_group_close(g);
      return BG_E_HIP;
    }
  }
  *out = g;
  return 0;
}

extern "C" int bg_group_open_rank(bg_group** out, int device, const void* uid, int nranks, int rank) {
  if (!out || !uid || nranks < 1 || rank < 0 || rank >= nranks) return BG_E_ARG;
  *out = nullptr;
  bg_group* g = new bg_group();
  bg_ctx* c = nullptr;
  int rc = bg_open(&c, device);
  if (rc) {
    delete g;
    return rc;
  }
  g->ctx.push_back(c);
  g->nranks = nranks;
  g->rank0 = rank;
  const char* se = getenv("BEDGPU_RCCL_SELF");
  g->self = nranks == 1 && se && strcmp(se, "0") != 0;
  if (nranks > 1 || g->self) {
    if (!rccl().ok) {
      group_warn("RCCL unavailable: " + rccl().err);
      bg_group_close(g);
      return BG_E_HIP;
    }
    ncclUniqueId id;
    if (g->self) {  // a one-rank group has no peer to share an id with
      const ncclResult_t ru = ncclGetUniqueId(&id);
      if (ru != ncclSuccess) {
        group_warn_nccl(ru, "ncclGetUniqueId");
        bg_group_close(g);
        return BG_E_HIP;
      }
    } else {
      memcpy(&id, uid, sizeof(id));
    }
    g->comm.resize(1);
    const ncclResult_t rr = ncclCommInitRank(&g->comm[0], nranks, id, rank);
    if (rr != ncclSuccess) {
      group_warn_nccl(rr, "ncclCommInitRank");
      g->comm.clear();
      bg_group_close(g);
      return BG_E_HIP;
    }
  }
  *out = g;
  return 0;
}

extern "C" int bg_group_size(const bg_group* g, int* nlocal, int* nranks, int* rank0) {
  if (!g) return BG_E_ARG;
  if (nlocal) *nlocal = (int)g->ctx.size();
  if (nranks) *nranks = g->nranks;
  if (rank0) *rank0 = g->rank0;
  return 0;
}

extern "C" bg_ctx* bg_group_ctx(bg_group* g, int k) {
  return (g && k >= 0 && k < (int)g->ctx.size()) ? g->ctx[k] : nullptr;
}

extern "C" void bg_group_close(bg_group* g) {
  if (!g) return;
  for (ncclComm_t c : g->comm) ncclCommDestroy(c);
  for (bg_ctx* c : g->ctx) bg_close(c);
  delete g;
}

// Reassemble the members' per-chromosome texts on global member 0.
// 1. totals: len[g] summed over members and owner[g] (+1) — ncclAllReduce of one
//    [2 x nchrom] uint64 array per member (host sums without communicators);
// 2. G[g] = exclusive prefix of len: chromosome g's place in the output;
// 3. every maximal run of consecutive chromosomes with one owner (zero-length ones
//    joined in) is one transfer: owner -> member 0, from the owner's text at off[first]
//    to out + G[first]; member 0's own runs are device copies. All sends and receives of
//    all local members go in one ncclGroupStart/End.
extern "C" int bg_group_gather(bg_group* g, int nchrom, const char* const* text,
                               const uint64_t* const* off, const uint64_t* const* len, char** out,
                               uint64_t* out_len) {
  if (!g || nchrom < 0 || !text || !off || !len || !out || !out_len) return BG_E_ARG;
  const int nl = (int)g->ctx.size();
  bg_ctx* c0 = g->ctx[0];
  *out = nullptr;
  *out_len = 0;
  const uint64_t nc = (uint64_t)nchrom;
  std::vector<uint64_t> tot(2 * nc, 0);  // [len..., owner+1...]
  if (g->comm.empty()) {
    for (int k = 0; k < nl; ++k)
      for (uint64_t q = 0; q < nc; ++q)
        if (len[k][q]) {
          tot[q] += len[k][q];
          tot[nc + q] = (uint64_t)(g->rank0 + k) + 1;
        }
  } else {
    std::vector<uint64_t*> dbuf(nl, nullptr);
    std::vector<uint64_t> h(2 * nc);
    // every exit below releases the size buffers, and a group that was started is ended
    auto release = [&]() {
      for (int k = 0; k < nl; ++k)
        if (dbuf[k]) {
          bg_bind(g->ctx[k]);
          hipStreamSynchronize(g->ctx[k]->stream);
          bg_release(g->ctx[k], dbuf[k]);
          dbuf[k] = nullptr;
        }
    };
    int rc = 0;
    for (int k = 0; k < nl && !rc; ++k) {
      bg_ctx* c = g->ctx[k];
      bg_bind(c);
      for (uint64_t q = 0; q < nc; ++q) {
        h[q] = len[k][q];
        h[nc + q] = len[k][q] ? (uint64_t)(g->rank0 + k) + 1 : 0;
      }
      dbuf[k] = (uint64_t*)bg_alloc(c, 16 * (nc ? nc : 1));
      if (!dbuf[k]) { rc = BG_E_NOMEM; break; }
      if (nc) rc = bg_hip_ok(c, hipMemcpyAsync(dbuf[k], h.data(), 16 * nc, hipMemcpyHostToDevice, c->stream));
      if (!rc) rc = bg_hip_ok(c, hipStreamSynchronize(c->stream));  // h is reused for the next member
    }
    if (!rc && nc) {
      ncclResult_t r = ncclGroupStart();
      const bool started = r == ncclSuccess;
      if (!started) rc = nccl_fail(c0, r, "ncclGroupStart");
      for (int k = 0; k < nl && !rc; ++k) {
        r = ncclAllReduce(dbuf[k], dbuf[k], 2 * nc, ncclUint64, ncclSum, g->comm[k], g->ctx[k]->stream);
        if (r != ncclSuccess) rc = nccl_fail(g->ctx[k], r, "ncclAllReduce");
      }
      if (started) {  // a started group is always ended
        const ncclResult_t e = ncclGroupEnd();
        if (!rc && e != ncclSuccess) rc = nccl_fail(c0, e, "ncclGroupEnd");
      }
    }
    if (!rc && nc) {
      bg_bind(c0);
      rc = bg_hip_ok(c0, hipMemcpyAsync(tot.data(), dbuf[0], 16 * nc, hipMemcpyDeviceToHost, c0->stream));
    }
    release();
    if (rc) return rc;
  }
  std::vector<uint64_t> G(nc + 1, 0);
  for (uint64_t q = 0; q < nc; ++q) G[q + 1] = G[q] + tot[q];
  const uint64_t total = G[nc];
  // runs of one owner
  struct Run { int owner; uint64_t first, bytes; };
  std::vector<Run> runs;
  for (uint64_t q = 0; q < nc; ++q) {
    if (!tot[q]) continue;
    const int own = (int)tot[nc + q] - 1;
    if (!runs.empty() && runs.back().owner == own) {
      runs.back().bytes += tot[q];
    } else {
      runs.push_back({own, q, tot[q]});
    }
  }
  const bool root = g->rank0 == 0;
  char* dst = nullptr;
  if (root) {
    bg_bind(c0);
    dst = (char*)bg_alloc(c0, total ? total : 1);
    if (!dst) return BG_E_NOMEM;
  }
  // device copies (member 0's own runs, and every run when there are no communicators)
  for (const Run& r : runs) {
    const int k = r.owner - g->rank0;
    if (k < 0 || k >= nl) continue;
    if (!root || (!g->comm.empty() && (r.owner != 0 || g->self))) continue;
    bg_ctx* c = g->ctx[k];
    bg_bind(c0);
    const void* src = text[k] + off[k][r.first];
    if (k == 0) BG_HIP(c0, hipMemcpyAsync(dst + G[r.first], src, r.bytes, hipMemcpyDeviceToDevice, c0->stream));
    else BG_HIP(c0, hipMemcpyPeerAsync(dst + G[r.first], c0->device, src, c->device, r.bytes, c0->stream));
  }
  if (!g->comm.empty()) {
    bool any = false;
    for (const Run& r : runs) any = any || r.owner != 0 || g->self;
    if (any) {
      int rc = 0;
      ncclResult_t e = ncclGroupStart();
      const bool started = e == ncclSuccess;
      if (!started) rc = nccl_fail(c0, e, "ncclGroupStart");
      for (size_t i = 0; i < runs.size() && !rc; ++i) {
        const Run& r = runs[i];
        if (r.owner == 0 && !g->self) continue;
        const int ks = r.owner - g->rank0;
        if (ks >= 0 && ks < nl) {
          e = ncclSend(text[ks] + off[ks][r.first], r.bytes, ncclChar, 0, g->comm[ks], g->ctx[ks]->stream);
          if (e != ncclSuccess) rc = nccl_fail(g->ctx[ks], e, "ncclSend");
        }
        if (!rc && root) {
          e = ncclRecv(dst + G[r.first], r.bytes, ncclChar, r.owner, g->comm[0], c0->stream);
          if (e != ncclSuccess) rc = nccl_fail(c0, e, "ncclRecv");
        }
      }
      if (started) {  // a started group is always ended
        const ncclResult_t z = ncclGroupEnd();
        if (!rc && z != ncclSuccess) rc = nccl_fail(c0, z, "ncclGroupEnd");
      }
      if (rc) {
        for (int k = 0; k < nl; ++k) {
          bg_bind(g->ctx[k]);
          hipStreamSynchronize(g->ctx[k]->stream);
        }
        if (dst) bg_release(c0, dst);
        return rc;
      }
    }
  }
  for (int k = 0; k < nl; ++k) {
    bg_bind(g->ctx[k]);
    BG_HIP(g->ctx[k], hipStreamSynchronize(g->ctx[k]->stream));
  }
  if (root) {
    *out = dst;
    *out_len = total;
  }
  return 0;
}

extern "C" void bg_device_free(bg_ctx* c, void* p) {
  if (!c || !p) return;
  bg_bind(c);
  hipStreamSynchronize(c->stream);
  bg_release(c, p);
}

// stream-ordered: the block returns to ctx's cache at once, and whatever reuses it is queued
// on ctx's stream after the work already there (no host wait)
extern "C" void bg_device_release(bg_ctx* c, void* p) {
  if (!c || !p) return;
  bg_release(c, p);
}

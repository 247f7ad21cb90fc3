// bg_api.hip — libbedgpu context, caching allocator, errors, result plumbing.
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>

#include "bg_internal.h"

// H2D / output staging slots of the ring (below): BEDGPU_RING_SLOTS (16; 16..64, rounded to a
// multiple of 16)
static int ring_slots() {
  static const int v = [] {
    const char* s = getenv("BEDGPU_RING_SLOTS");
    const int n = s ? atoi(s) : 16;
    return n < 16 ? 16 : (n > 64 ? 64 : n / 16 * 16);
  }();
  return v;
}
#define BG_RING_SLOTS ring_slots()
#define BG_WR_SLOTS 8     // after the ring's slots: the output queue's (bg_writer)

static int ring_threads();
static void pool_start(bg_ctx* c, int n);
void bg_pool_stop(bg_ctx* c);

int bg_fail(bg_ctx* c, int code, const std::string& msg) {
  if (!c) return code;
  if (std::this_thread::get_id() != c->owner) {
    std::lock_guard<std::mutex> g(c->copy_mu);
    c->err_async = msg;
    return code;
  }
  c->err = msg;
  return code;
}

int bg_hip_fail(bg_ctx* c, hipError_t e, const char* what) {
  std::string m = std::string("HIP error: ") + hipGetErrorString(e) + " in " + what;
  if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return bg_fail(c, BG_E_NOMEM, m);
  return bg_fail(c, BG_E_HIP, m);
}

void* bg_alloc(bg_ctx* c, size_t bytes) {
  bg_bind(c);  // the calling thread may drive several devices (bg_group)
  bytes = (bytes + 255) & ~(size_t)255;
  if (bytes == 0) bytes = 256;
  // best fit among cached blocks no larger than 2x the request
  size_t best = (size_t)-1;
  for (size_t k = 0; k < c->free_list.size(); ++k) {
    const size_t b = c->free_list[k].bytes;
    if (b >= bytes && b <= 2 * bytes && (best == (size_t)-1 || b < c->free_list[best].bytes)) best = k;
  }
  void* p = nullptr;
  size_t got = bytes;
  if (best != (size_t)-1) {
    p = c->free_list[best].p;
    got = c->free_list[best].bytes;
    c->free_list.erase(c->free_list.begin() + best);
  } else {
    const auto ta = std::chrono::steady_clock::now();
    const hipError_t me = hipMalloc(&p, bytes);
    if (c->stats) {
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ta).count();
      if (ms > 2.0) fprintf(stderr, "bedgpu alloc %.1f MB took %.1f ms\n", bytes / 1e6, ms);
    }
    if (me != hipSuccess) {
      (void)hipGetLastError();
      // drop the cache and retry once
      hipStreamSynchronize(c->stream);
      if (c->sstream) hipStreamSynchronize(c->sstream);
      for (auto& b : c->free_list) hipFree(b.p);
      c->free_list.clear();
      if (hipMalloc(&p, bytes) != hipSuccess) {
        (void)hipGetLastError();
        bg_fail(c, BG_E_NOMEM, "device allocation of " + std::to_string(bytes) + " bytes failed");
        return nullptr;
      }
    }
  }
  c->live[p] = got;
  return p;
}

void bg_release(bg_ctx* c, void* p) {
  if (!c || !p) return;
  auto& L = c->live;
  auto it = L.find(p);
  if (it == L.end()) return;
  (c->defer_release ? c->deferred : c->free_list).push_back({p, it->second});
  L.erase(it);
}

void bg_mark(bg_ctx* c, const char* name) {
  if (!c->stats) return;
  hipEvent_t ev;
  if (hipEventCreate(&ev) != hipSuccess) return;
  hipEventRecord(ev, c->stream);
  c->marks.emplace_back(name, ev);
}

bool bg_prof_on(bg_ctx* c, const char* name) {
  if (c->prof_filter.empty()) return false;
  return c->prof_filter == "*" || c->prof_filter == name;
}

hipEvent_t bg_prof_event(bg_ctx* c) {
  if (!c->prof_events.empty()) {
    hipEvent_t e = c->prof_events.back();
    c->prof_events.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

void bg_prof_push(bg_ctx* c, const char* name, hipEvent_t a, hipEvent_t b) {
  c->prof_pending.push_back({name, a, b});
  if (c->prof_pending.size() > 4096) {  // bound the number of live events
    (void)hipStreamSynchronize(c->stream);
    char tmp[8];
    bg_prof_read(c, tmp, 0);
  }
}

static void prof_drain(bg_ctx* c) {
  if (c->prof_pending.empty()) return;
  (void)hipStreamSynchronize(c->stream);
  for (auto& p : c->prof_pending) {
    float ms = 0;
    (void)hipEventElapsedTime(&ms, p.a, p.b);
    size_t k = 0;
    while (k < c->prof.size() && c->prof[k].first != p.name) ++k;
    if (k == c->prof.size()) c->prof.push_back({p.name, bg_ctx::KStat()});
    c->prof[k].second.ms += ms;
    c->prof[k].second.calls += 1;
    c->prof_events.push_back(p.a);
    c->prof_events.push_back(p.b);
  }
  c->prof_pending.clear();
}

// filter: NULL or "" disables, "*" profiles every kernel, else one kernel name.
// Enabling clears the accumulated statistics.
extern "C" int bg_prof_enable(bg_ctx* c, const char* filter) {
  if (!c) return BG_E_ARG;
  prof_drain(c);
  c->prof.clear();
  c->prof_filter = filter ? filter : "";
  return 0;
}

// "name calls total_ms" lines, one per kernel, in first-launch order
extern "C" int bg_prof_read(bg_ctx* c, char* buf, uint64_t cap) {
  if (!c) return BG_E_ARG;
  prof_drain(c);
  if (!buf || cap == 0) return 0;
  std::string s;
  for (auto& kv : c->prof) {
    char line[256];
    snprintf(line, sizeof(line), "%s %llu %.6f\n", kv.first.c_str(),
             (unsigned long long)kv.second.calls, kv.second.ms);
    s += line;
  }
  snprintf(buf, cap, "%s", s.c_str());
  return 0;
}

void bg_ring_start(bg_ctx* c);
extern "C" int bg_open(bg_ctx** out, int device) {
  if (!out) return BG_E_ARG;
  *out = nullptr;
  bg_ctx* c = new bg_ctx();
  c->owner = std::this_thread::get_id();
  c->device = device;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    (void)hipGetLastError();  // not sticky: a later context's checks must not see it
    delete c;
    return BG_E_HIP;
  }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&c->dstat, sizeof(bg_dstatus)) != hipSuccess || hipMalloc(&c->warm, 16u << 20) != hipSuccess ||
      hipHostMalloc(&c->hstat, sizeof(bg_dstatus), hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    delete c;
    return BG_E_HIP;
  }
  if (hipDeviceGetAttribute(&c->ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    c->ncu = 256;
  const char* st = getenv("BEDGPU_STATS");
  c->stats = st && *st && strcmp(st, "0") != 0;
  bg_ring_start(c);
  bg_mark(c, "open");
  *out = c;
  return 0;
}

extern "C" void bg_close(bg_ctx* c) {
  if (!c) return;
  if (c->ring_th.joinable()) c->ring_th.join();
  bg_pool_stop(c);
  hipStreamSynchronize(c->stream);
  if (c->sstream) hipStreamSynchronize(c->sstream);
  for (auto& b : c->free_list) hipFree(b.p);
  for (auto& b : c->deferred) hipFree(b.p);
  for (auto& kv : c->live) hipFree(kv.first);
  for (auto& m : c->marks) hipEventDestroy(m.second);
  for (auto& p : c->prof_pending) { hipEventDestroy(p.a); hipEventDestroy(p.b); }
  for (auto e : c->prof_events) hipEventDestroy(e);
  hipFree(c->dstat);
  hipFree(c->warm);
  hipHostFree(c->hstat);
  for (auto& ch : c->pin_chunks) hipHostFree(ch.first);
  for (auto e : c->ring_ev)
    if (e) hipEventDestroy(e);
  for (size_t k = c->ring_base ? BG_RING_SLOTS : 0; k < c->ring.size(); ++k)
    if (c->ring[k]) hipHostFree(c->ring[k]);
  if (c->ring_base) hipHostFree(c->ring_base);
  if (c->pstream) hipStreamSynchronize(c->pstream);
  for (auto e : c->copy_ev) hipEventDestroy(e);
  for (auto e : c->order_ev) hipEventDestroy(e);
  if (c->pstream) hipStreamDestroy(c->pstream);
  if (c->sstream) hipStreamDestroy(c->sstream);
  if (c->sfork) hipEventDestroy(c->sfork);
  if (c->sjoin) hipEventDestroy(c->sjoin);
  hipStreamDestroy(c->stream);
  delete c;
}

void bg_pin_reset(bg_ctx* c) {
  c->pin_chunk = 0;
  c->pin_used = 0;
}

void* bg_pin_take(bg_ctx* c, size_t bytes) {
  bytes = (bytes + 63) & ~(size_t)63;
  while (c->pin_chunk < c->pin_chunks.size()) {
    auto& ch = c->pin_chunks[c->pin_chunk];
    if (c->pin_used + bytes <= ch.second) {
      void* p = ch.first + c->pin_used;
      c->pin_used += bytes;
      return p;
    }
    ++c->pin_chunk;
    c->pin_used = 0;
  }
  const size_t sz = std::max<size_t>(bytes, 4u << 20);
  char* p = nullptr;
  if (hipHostMalloc((void**)&p, sz, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  c->pin_chunks.push_back({p, sz});
  c->pin_chunk = c->pin_chunks.size() - 1;
  c->pin_used = bytes;
  return p;
}

uint32_t bg_resident_blocks(bg_ctx* c, const void* kern) {
  for (auto& kv : c->resident)
    if (kv.first == kern) return kv.second;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, BG_NT, 0) != hipSuccess || per_cu < 1)
    per_cu = 1;
  const uint32_t n = (uint32_t)per_cu * (uint32_t)c->ncu;
  c->resident.push_back({kern, n});
  return n;
}

extern "C" const char* bg_last_error(const bg_ctx* c) {
  if (!c) return "no context";
  bg_ctx* m = const_cast<bg_ctx*>(c);
  {
    std::lock_guard<std::mutex> g(m->copy_mu);
    if (!m->err_async.empty()) {
      m->err = m->err_async;
      m->err_async.clear();
    }
  }
  return m->err.c_str();
}

extern "C" int bg_sync(bg_ctx* c) {
  BG_HIP(c, hipStreamSynchronize(c->stream));
  return 0;
}

extern "C" void* bg_stream(bg_ctx* c) { return c ? (void*)c->stream : nullptr; }

extern "C" int bg_stats(const bg_ctx* cc, char* buf, uint64_t cap) {
  bg_ctx* c = const_cast<bg_ctx*>(cc);
  if (!c || !buf || !cap) return BG_E_ARG;
  std::string s;
  hipStreamSynchronize(c->stream);
  for (size_t k = 1; k < c->marks.size(); ++k) {
    float ms = 0;
    hipEventElapsedTime(&ms, c->marks[k - 1].second, c->marks[k].second);
    char line[128];
    snprintf(line, sizeof(line), "bedgpu stage %-12s %10.3f ms\n", c->marks[k].first.c_str(), ms);
    s += line;
  }
  snprintf(buf, cap, "%s", s.c_str());
  return 0;
}

extern "C" int bg_set_restrict_chrom(bg_ctx* c, bg_set* s, const char* chrom) {
  if (!c || !s || !chrom) return BG_E_ARG;
  for (bg_table* T : s->t)
    if (T->is_set) return bg_fail(c, BG_E_ARG, "--chrom: an input was loaded as BG_BED3_SET (no rows kept)");
  for (bg_table* T : s->t) {
    uint64_t a = 0, b = 0;
    for (size_t k = 0; k + 1 < T->run_row0.size(); ++k)
      if (T->run_name[k] == chrom) { a = T->run_row0[k]; b = T->run_row0[k + 1]; }
    const uint64_t n = b - a;
    auto sub = [&](void* p, size_t w) -> void* {
      if (!p) return nullptr;
      void* q = bg_alloc(c, w * (n ? n : 1));
      if (q && n) hipMemcpyAsync(q, (char*)p + w * a, w * n, hipMemcpyDeviceToDevice, c->stream);
      bg_release(c, p);
      return q;
    };
    T->ks = (int64_t*)sub(T->ks, 8);
    T->ke = (int64_t*)sub(T->ke, 8);
    T->rest_off = (uint64_t*)sub(T->rest_off, 8);
    T->rest_len = (uint32_t*)sub(T->rest_len, 4);
    T->score = (double*)sub(T->score, 8);
    T->n = n;
    T->run_row0.assign({0, n});
    T->run_name.assign({std::string(chrom)});
    if (!T->ks || !T->ke) return BG_E_NOMEM;
  }
  return 0;
}

extern "C" int bg_result_rows(const bg_result* r, uint64_t* rows) {
  if (!r || !rows) return BG_E_ARG;
  if (r->n_pending) {  // a segmented result's count is fetched on first use
    bg_result* w = const_cast<bg_result*>(r);
    const int rc = bg_result_resolve_n(w->ctx, w);
    if (rc) return rc;
  }
  *rows = r->n;
  return 0;
}

extern "C" int bg_result_text_device(const bg_result* r, const char** dptr, uint64_t* nbytes) {
  if (!r || !dptr || !r->formatted) return BG_E_ARG;
  *dptr = r->text;
  if (nbytes) *nbytes = r->nbytes;
  return 0;
}

extern "C" int bg_result_copy_text(bg_ctx* c, bg_result* r, char* host, uint64_t cap) {
  uint64_t n = 0;
  int rc = bg_result_format(c, r, &n);
  if (rc && rc != BG_E_VISITOR) return rc;  // BG_E_VISITOR: the text before the stop
  if (cap < n) return bg_fail(c, BG_E_ARG, "host buffer too small");
  if (n) BG_HIP(c, hipMemcpyAsync(host, r->text, n, hipMemcpyDeviceToHost, c->stream));
  BG_HIP(c, hipStreamSynchronize(c->stream));
  return rc;
}


// ---------------------------------------------------------------------------------------
// Input files -> HBM. A file is mapped read-only with its page-cache pages faulted in
// (MAP_POPULATE: page-table entries only, no copy, no GPU call, so the front-ends run it
// while bg_open initialises HIP); after that, threads copy it from the page cache into a
// driver-pinned staging ring whose slots the DMA engines stream to HBM (ring_h2d below).
// What was measured on the box and dropped (tools/e2e_probe.cpp, tools/gpu_e2e_r03.sh):
//   - registering the mapping (or an anonymous copy of it) with hipHostRegister and DMA-ing
//     straight from it: fast in isolation (register 5-19 ms, copy ~45 ms per 2.38 GB) but
//     inside the CLI the first kernels stalled by 250-450 ms;
//   - reading the file into anonymous memory during HIP init: freeing 2.38 GB of 4 KiB
//     pages afterwards costs ~240 ms (munmap, or the same at process exit);
//   - the round-2 pread ring: needed extra copy streams (8-40 ms each to create, more to
//     tear down at exit) and could not start before HIP was up.
// ---------------------------------------------------------------------------------------
// BEDGPU_RD_PREAD=1: a file image's chunks are read into the slots with pread(2) (the kernel
// copies from the page cache; no page faults on the mapping) instead of memcpy from the mapping
static bool rd_pread() {
  static const bool v = [] {
    const char* s = getenv("BEDGPU_RD_PREAD");
    return s && strcmp(s, "1") == 0;
  }();
  return v;
}
// open files of the images (pread sources, BEDGPU_RD_PREAD), by mapping address
static std::mutex img_mu;
static std::unordered_map<const char*, int> img_fd;
static int image_fd(const bg_file_image* m) {
  std::lock_guard<std::mutex> g(img_mu);
  auto it = img_fd.find(m->data);
  return it == img_fd.end() ? -1 : it->second;
}

extern "C" int bg_file_image_open(const char* path, bg_file_image* m) {
  if (!path || !m) return BG_E_ARG;
  memset(m, 0, sizeof(*m));
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return BG_E_IO;
  struct stat st;
  if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode)) {
    close(fd);
    return BG_E_ARG;
  }
  m->n = (uint64_t)st.st_size;
  if (m->n) {
    // BEDGPU_POPULATE=1: fault the page-table entries in here (MAP_POPULATE). Off by default:
    // populating holds the mm's lock for the whole file and HIP's initialisation (its own
    // mappings) waited on it — bg_open 135-155 ms instead of ~80 ms on the box, with the
    // copies no faster (gpurun_out/e2e_var, profiles/r03_e2e_var.txt)
    static const bool populate = [] {
      const char* s = getenv("BEDGPU_POPULATE");
      return s && strcmp(s, "1") == 0;
    }();
    void* p = mmap(nullptr, (size_t)m->n, PROT_READ, MAP_SHARED | (populate ? MAP_POPULATE : 0), fd, 0);
    if (p == MAP_FAILED) {
      close(fd);
      m->n = 0;
      return BG_E_IO;
    }
    m->data = (const char*)p;
    if (rd_pread()) {
      std::lock_guard<std::mutex> g(img_mu);
      img_fd[m->data] = fd;
      return 0;
    }
  }
  close(fd);
  return 0;
}

// The staging ring: BG_RING_SLOTS driver-pinned slots of BG_RING_CH bytes with one event
// each, allocated on first use by as many threads (hipHostMalloc of a few MiB costs 5-25 ms
// per call on the box). Host memory registered with hipHostRegister is avoided for bulk
// copies: in the CLI, kernels running while registered (user-pointer) pages of the input
// images or of output bounce buffers were in use stalled by 250-450 ms per run (the driver
// evicts and restores the queues when such pages are invalidated); the ring's pages are the
// driver's own.
// slot bytes: BEDGPU_RING_MB (1..16, default 2); pinning cost grows with the slot size
static uint64_t ring_ch() {
  static const uint64_t v = [] {
    const char* s = getenv("BEDGPU_RING_MB");
    const long m = s ? atol(s) : 2;
    return (uint64_t)(m < 1 ? 1 : (m > 16 ? 16 : m)) << 20;
  }();
  return v;
}
#define BG_RING_CH ring_ch()
// H2D chunks per DMA: BEDGPU_RING_GROUP (1, 2, 4, 8 or 16; default 4). The threads fill
// BG_RING_CH chunks, the last filler of a group of consecutive chunks issues ONE copy for
// the group: measured on the box (tools/h2d_probe.py, profiles/r04_h2d_probe.txt) 2 MiB
// copies run at ~40 GB/s, 8 MiB and larger at ~57 GB/s
static int ring_group() {
  static const int v = [] {
    const char* s = getenv("BEDGPU_RING_GROUP");
    const int g = s ? atoi(s) : 4;
    return (g == 1 || g == 2 || g == 4 || g == 8 || g == 16) ? g : 4;
  }();
  return v;
}
static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// pins the ring's slots, one thread each (bg_open runs this on a thread of its own, so the
// pinning overlaps whatever the caller does next)
// slot events wait by sleeping (hipEventBlockingSync) instead of polling, leaving the
// box's CPU quota (16 CPUs) to the copying threads and the output writer; the copies are
// DMA-bound either way (profiles/r03_e2e/var_i5_summary.txt). BEDGPU_EVENT_BLOCK=0: poll
static bool event_block() {
  static const bool v = [] {
    const char* s = getenv("BEDGPU_EVENT_BLOCK");
    return !(s && strcmp(s, "0") == 0);
  }();
  return v;
}
static int ring_alloc(bg_ctx* c) {
  const double t0 = now_ms();
  std::vector<char*> ring(BG_RING_SLOTS + BG_WR_SLOTS, nullptr);
  std::vector<hipEvent_t> ev(BG_RING_SLOTS + BG_WR_SLOTS, nullptr);
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  static const bool warm = [] {  // BEDGPU_RING_WARM=0: no warm-up copy
    const char* s = getenv("BEDGPU_RING_WARM");
    return !(s && strcmp(s, "0") == 0);
  }();
  // the H2D slots in ONE allocation, so that consecutive slots take one DMA (ring_h2d's
  // groups); the output slots one allocation each
  const bool one = ring_group() > 1;
  char* base = nullptr;
  for (int k = 0; k < BG_RING_SLOTS + BG_WR_SLOTS; ++k)
    th.emplace_back([&, k]() {
      char** dst = &ring[k];
      size_t bytes = BG_RING_CH;
      if (one && k < BG_RING_SLOTS) {
        dst = k == 0 ? &base : nullptr;
        bytes = (size_t)BG_RING_SLOTS * BG_RING_CH;
      }
      if (hipSetDevice(c->device) != hipSuccess ||
          (dst && hipHostMalloc((void**)dst, bytes, hipHostMallocDefault) != hipSuccess) ||
          hipEventCreateWithFlags(&ev[k], hipEventDisableTiming | (event_block() ? hipEventBlockingSync : 0)) !=
              hipSuccess) {
        bad = 1;
        return;
      }
      // the runtime's first host->device copy on the stream costs ~15 ms more than the
      // next ones (measured): take it here, while the other slots are being pinned
      if (k == 0 && warm && c->warm)  // a full slot: small copies take another path (blit kernel)
        (void)hipMemcpyAsync(c->warm, one ? base : ring[0], BG_RING_CH, hipMemcpyHostToDevice, c->stream);
    });
  for (auto& x : th) x.join();
  if (bad) {
    (void)hipGetLastError();
    for (auto e : ev)
      if (e) hipEventDestroy(e);
    for (auto p : ring)
      if (p) hipHostFree(p);
    if (base) hipHostFree(base);
    return BG_E_HIP;
  }
  if (one)
    for (int k = 0; k < BG_RING_SLOTS; ++k) ring[k] = base + (size_t)k * BG_RING_CH;
  c->ring_base = base;
  c->ring = ring;
  c->ring_ev = ev;
  pool_start(c, ring_threads() - 1);
  if (c->stats)
    fprintf(stderr, "bedgpu ring   %d x %llu MiB pinned in %.3f ms\n", (int)(BG_RING_SLOTS + BG_WR_SLOTS),
            (unsigned long long)(BG_RING_CH >> 20), now_ms() - t0);
  return 0;
}
void bg_ring_start(bg_ctx* c) {
  c->ring_th = std::thread([c]() { c->ring_rc = ring_alloc(c); });
}
static int ring_get(bg_ctx* c) {
  if (c->ring_th.joinable()) c->ring_th.join();
  if (!c->ring.empty()) return 0;
  if (c->ring_rc == 0) c->ring_rc = ring_alloc(c);  // not started, or an earlier attempt failed
  if (c->ring_rc) {
    c->ring_rc = 0;  // a later call may retry
    return bg_fail(c, BG_E_HIP, "staging ring");
  }
  return 0;
}

// host -> device through the ring: T threads copy chunks of `src` into their slots (CPU
// memcpy from cached pages) and queue the slot's DMA on ctx's stream, reusing a slot once its
// event says the previous DMA out of it has completed
// (BEDGPU_RING_THREADS: 1..16, default 8: the copies are DMA-bound, threads wait ~80% of
// the time with 16)
static int ring_threads() {
  static const int t = [] {
    const char* s = getenv("BEDGPU_RING_THREADS");
    const int v = s ? atoi(s) : 8;
    return v < 1 ? 1 : (v > BG_RING_SLOTS ? BG_RING_SLOTS : v);
  }();
  return t;
}
// (Measured and removed in round 6: a second copy stream, and kernels pulling the pinned
// slots over the link instead of the DMA engine — the same 38-44 GB/s)
// The ring's copy threads: started once with the ring (bg_open's thread), parked on a
// condition variable between calls. (Spawning them per call cost 4-7 ms the first time:
// thread stacks mapped while HIP was mapping its own memory.)
struct bg_pool {
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable go, done;
  const std::function<void(int)>* job = nullptr;
  uint64_t gen = 0;
  int pending = 0;
  bool stop = false;
};
static void pool_start(bg_ctx* c, int n) {
  bg_pool* P = new bg_pool();
  c->pool = P;
  for (int t = 1; t <= n; ++t)
    P->th.emplace_back([c, P, t]() {
      (void)hipSetDevice(c->device);
      uint64_t seen = 0;
      for (;;) {
        const std::function<void(int)>* job;
        {
          std::unique_lock<std::mutex> g(P->mu);
          P->go.wait(g, [&] { return P->stop || P->gen != seen; });
          if (P->stop) return;
          seen = P->gen;
          job = P->job;
        }
        (*job)(t);
        std::lock_guard<std::mutex> g(P->mu);
        if (--P->pending == 0) P->done.notify_all();
      }
    });
}
static void pool_run(bg_ctx* c, const std::function<void(int)>& job) {
  bg_pool* P = c->pool;
  if (!P) {  // no pool (not started): run every share here
    for (int t = 0; t < 16; ++t) job(t);
    return;
  }
  {
    std::lock_guard<std::mutex> g(P->mu);
    P->job = &job;
    P->pending = (int)P->th.size();
    ++P->gen;
  }
  P->go.notify_all();
  job(0);
  std::unique_lock<std::mutex> g(P->mu);
  P->done.wait(g, [&] { return P->pending == 0; });
}
void bg_pool_stop(bg_ctx* c) {
  bg_pool* P = c->pool;
  if (!P) return;
  {
    std::lock_guard<std::mutex> g(P->mu);
    P->stop = true;
  }
  P->go.notify_all();
  for (auto& x : P->th) x.join();
  delete P;
  c->pool = nullptr;
}
// one chunk of the source into a ring slot (memcpy from the mapping, or pread)
static bool ring_fill(char* slot, const char* src, uint64_t off, uint64_t len, int fd, uint64_t foff) {
  if (fd < 0) {
    memcpy(slot, src + off, len);
    return true;
  }
  uint64_t got = 0;
  while (got < len) {
    const ssize_t r = pread(fd, slot + got, len - got, (off_t)(foff + off + got));
    if (r <= 0) {
      if (r < 0 && errno == EINTR) continue;
      return false;
    }
    got += (uint64_t)r;
  }
  return true;
}

// ring_h2d with G chunks per DMA: chunk k lives in slot (k / G % (SLOTS / G)) * G + k % G, so a
// group's chunks are contiguous; the thread that completes a group issues its copy and
// records the group slot's event. A thread refills a group slot only after the group that
// used it before was issued (subm) and its copy completed (the event).
static int ring_h2d_grouped(bg_ctx* c, char* dst, const char* src, uint64_t n, int fd, uint64_t foff, int G,
                            hipStream_t cs) {
  const uint64_t CH = BG_RING_CH, nch = (n + CH - 1) / CH, ngr = (nch + G - 1) / G;
  const int NGS = BG_RING_SLOTS / G;
  const int T = (int)std::min<uint64_t>(ring_threads(), nch);
  std::mutex mu;
  std::condition_variable cv;
  std::vector<int64_t> subm(NGS, -1);  // the last group issued from each group slot (this call)
  std::unique_ptr<std::atomic<uint32_t>[]> filled(new std::atomic<uint32_t>[ngr]);
  for (uint64_t g = 0; g < ngr; ++g) filled[g] = 0;
  std::atomic<int> bad{0};
  std::atomic<int64_t> t_wait{0}, t_copy{0};
  auto worker = [&](int t) {
    if (hipSetDevice(c->device) != hipSuccess) { bad = 1; cv.notify_all(); return; }
    for (uint64_t k = (uint64_t)t; k < nch && !bad; k += (uint64_t)T) {
      const uint64_t gk = k / G;
      const int gs = (int)(gk % NGS), sl = gs * G + (int)(k % G);
      const auto a0 = std::chrono::steady_clock::now();
      if (gk >= (uint64_t)NGS) {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return subm[gs] >= (int64_t)(gk - NGS) || bad; });
        if (bad) return;
      }
      if (hipEventSynchronize(c->ring_ev[gs * G]) != hipSuccess) { bad = 1; cv.notify_all(); return; }
      const uint64_t off = k * CH, len = std::min<uint64_t>(CH, n - off);
      const auto a1 = std::chrono::steady_clock::now();
      if (!ring_fill(c->ring[sl], src, off, len, fd, foff)) { bad = 1; cv.notify_all(); return; }
      if (c->stats) {
        const auto a2 = std::chrono::steady_clock::now();
        t_wait += std::chrono::duration_cast<std::chrono::nanoseconds>(a1 - a0).count();
        t_copy += std::chrono::duration_cast<std::chrono::nanoseconds>(a2 - a1).count();
      }
      const uint32_t in_group = (uint32_t)std::min<uint64_t>(G, nch - gk * G);
      if (filled[gk].fetch_add(1) + 1 == in_group) {  // the group is complete: one copy
        const uint64_t go = gk * G * CH, glen = std::min<uint64_t>((uint64_t)G * CH, n - go);
        std::lock_guard<std::mutex> g(mu);
        if (hipMemcpyAsync(dst + go, c->ring[gs * G], glen, hipMemcpyHostToDevice, cs) != hipSuccess ||
            hipEventRecord(c->ring_ev[gs * G], cs) != hipSuccess)
          bad = 1;
        subm[gs] = (int64_t)gk;
        cv.notify_all();
      }
    }
  };
  const double t0 = now_ms();
  const std::function<void(int)> job = [&](int t) {
    if (t < T) worker(t);
  };
  pool_run(c, job);
  if (c->stats) {
    const double t1 = now_ms();
    hipStreamSynchronize(cs);
    fprintf(stderr, "bedgpu ring   %.1f MB: copies issued %.3f ms, drained %.3f ms (threads: %.1f ms waiting, %.1f ms copying; %d chunks per copy)\n",
            n / 1e6, t1 - t0, now_ms() - t0, t_wait / 1e6, t_copy / 1e6, G);
  }
  return bad ? bg_fail(c, BG_E_HIP, "staging ring copy") : 0;
}

// fd >= 0: src is the mapping of that file at offset foff (pread source when rd_pread())
static int ring_h2d(bg_ctx* c, char* dst, const char* src, uint64_t n, int fd = -1, uint64_t foff = 0) {
  if (!n) return 0;
  int rc = ring_get(c);
  if (rc) return rc;
  if (c->ring_base)
    return ring_h2d_grouped(c, dst, src, n, fd, foff, ring_group(), c->stream);
  const uint64_t nch = (n + BG_RING_CH - 1) / BG_RING_CH;
  const int TT_ = ring_threads();
  const int T = (int)std::min<uint64_t>(TT_, nch);
  const int per = BG_RING_SLOTS / TT_;  // slots per thread
  std::mutex mu;
  std::atomic<int> bad{0};
  std::atomic<int64_t> t_wait{0}, t_copy{0};  // stats: ns in event waits / memcpy, all threads
  auto worker = [&](int t) {
    if (hipSetDevice(c->device) != hipSuccess) { bad = 1; return; }
    uint64_t j = 0;
    for (uint64_t k = (uint64_t)t; k < nch && !bad; k += (uint64_t)T, ++j) {
      const int sl = t * per + (int)(j % per);
      const auto a0 = std::chrono::steady_clock::now();
      if (hipEventSynchronize(c->ring_ev[sl]) != hipSuccess) { bad = 1; return; }
      const uint64_t off = k * BG_RING_CH, len = std::min<uint64_t>(BG_RING_CH, n - off);
      const auto a1 = std::chrono::steady_clock::now();
      if (fd >= 0) {
        uint64_t got = 0;
        while (got < len) {
          const ssize_t r = pread(fd, c->ring[sl] + got, len - got, (off_t)(foff + off + got));
          if (r <= 0) {
            if (r < 0 && errno == EINTR) continue;
            bad = 1;
            return;
          }
          got += (uint64_t)r;
        }
      } else {
        memcpy(c->ring[sl], src + off, len);
      }
      if (c->stats) {
        const auto a2 = std::chrono::steady_clock::now();
        t_wait += std::chrono::duration_cast<std::chrono::nanoseconds>(a1 - a0).count();
        t_copy += std::chrono::duration_cast<std::chrono::nanoseconds>(a2 - a1).count();
      }
      std::lock_guard<std::mutex> g(mu);
      if (hipMemcpyAsync(dst + off, c->ring[sl], len, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
          hipEventRecord(c->ring_ev[sl], c->stream) != hipSuccess) {
        bad = 1;
        return;
      }
    }
  };
  const double t0 = now_ms();
  const std::function<void(int)> job = [&](int t) {
    if (t < T) worker(t);
  };
  pool_run(c, job);  // the pool's threads take t = 1..; this thread t = 0
  const double t_spawn = now_ms();
  if (c->stats) {  // the last copies drained (stats runs only: this waits)
    const double t1 = now_ms();
    hipStreamSynchronize(c->stream);
    fprintf(stderr, "bedgpu ring   %.1f MB: copies issued %.3f ms, drained %.3f ms (threads: %.1f ms waiting, %.1f ms copying; spawn %.3f ms)\n",
            n / 1e6, t1 - t0, now_ms() - t0, t_wait / 1e6, t_copy / 1e6, t_spawn - t0);
  }
  return bad ? bg_fail(c, BG_E_HIP, "staging ring copy") : 0;
}

// BEDGPU_IMG_COPY=reg: register the image and DMA from it; =pageable: the runtime's own
// staging; default: through the ring (above)
static int img_copy_mode() {
  static const int m = [] {
    const char* s = getenv("BEDGPU_IMG_COPY");
    if (s && !strcmp(s, "reg")) return 1;
    if (s && !strcmp(s, "pageable")) return 2;
    return 0;
  }();
  return m;
}

extern "C" int bg_file_image_register(bg_file_image* m) {
  if (!m) return BG_E_ARG;
  if (m->registered || !m->n || img_copy_mode() != 1) return 0;
  if (hipHostRegister((void*)m->data, (size_t)m->n, hipHostRegisterPortable) != hipSuccess) {
    (void)hipGetLastError();
    return BG_E_HIP;  // the copies still work (pageable source), staged by the runtime
  }
  m->registered = 1;
  return 0;
}

extern "C" int bg_file_image_to_device(bg_ctx* c, const bg_file_image* m, uint64_t off, uint64_t len, void** out) {
  if (!c || !m || !out || off > m->n || len > m->n - off) return BG_E_ARG;
  *out = nullptr;
  bg_bind(c);
  char* d = (char*)bg_alloc(c, len + 64);
  if (!d) return BG_E_NOMEM;
  int rc = 0;
  if (len) {
    if (m->registered || img_copy_mode() == 2) {
      const hipError_t e = hipMemcpyAsync(d, m->data + off, (size_t)len, hipMemcpyHostToDevice, c->stream);
      if (e != hipSuccess) rc = bg_hip_fail(c, e, "file image copy");
    } else {
      const int fd = rd_pread() ? image_fd(m) : -1;
      rc = ring_h2d(c, d, m->data + off, len, fd, off);
    }
  }
  if (rc) {
    hipStreamSynchronize(c->stream);
    bg_release(c, d);
    return rc;
  }
  *out = d;
  return 0;
}

// prefetch copies: issued by a host thread of the caller's on the context's prefetch stream
// while ctx's stream runs earlier groups' kernels; bg_copy_fence orders ctx's stream after a
// slot's copies (the caller's thread that launches kernels calls it, once the copy was issued)
extern "C" int bg_device_alloc(bg_ctx* c, uint64_t n, void** out) {
  if (!c || !out) return BG_E_ARG;
  bg_bind(c);
  *out = bg_alloc(c, n ? n : 1);
  return *out ? 0 : BG_E_NOMEM;
}

extern "C" int bg_file_image_copy(bg_ctx* c, const bg_file_image* m, uint64_t off, uint64_t len, void* dst,
                                  int slot) {
  if (!c || !m || !dst || slot < 0 || slot >= 65536 || off > m->n || len > m->n - off) return BG_E_ARG;
  bg_bind(c);
  hipStream_t ps = nullptr;
  hipEvent_t ev = nullptr;
  {
    std::lock_guard<std::mutex> g(c->copy_mu);
    if (!c->pstream && hipStreamCreateWithFlags(&c->pstream, hipStreamNonBlocking) != hipSuccess) {
      c->pstream = nullptr;
      return BG_E_HIP;
    }
    while ((int)c->copy_ev.size() <= slot) {
      hipEvent_t e = nullptr;
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return BG_E_HIP;
      c->copy_ev.push_back(e);
    }
    ps = c->pstream;
    ev = c->copy_ev[slot];
    // the destination may be a block ctx's stream used before (the caching allocator):
    // the copies start after the position bg_copy_order recorded for this slot
    if (slot < (int)c->order_set.size() && c->order_set[slot] &&
        hipStreamWaitEvent(ps, c->order_ev[slot], 0) != hipSuccess)
      return BG_E_HIP;
  }
  int rc = 0;
  if (len) {
    if ((rc = ring_get(c))) return rc;
    if (c->ring_base) {
      const int fd = rd_pread() ? image_fd(m) : -1;
      rc = ring_h2d_grouped(c, (char*)dst, m->data + off, len, fd, off, ring_group(), ps);
    } else if (hipMemcpyAsync(dst, m->data + off, (size_t)len, hipMemcpyHostToDevice, ps) != hipSuccess) {
      rc = BG_E_HIP;
    }
  }
  if (!rc && hipEventRecord(ev, ps) != hipSuccess) rc = BG_E_HIP;
  return rc;
}

extern "C" int bg_copy_order(bg_ctx* c, int slot) {
  if (!c || slot < 0 || slot >= 65536) return BG_E_ARG;
  bg_bind(c);
  std::lock_guard<std::mutex> g(c->copy_mu);
  while ((int)c->order_ev.size() <= slot) {
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return BG_E_HIP;
    c->order_ev.push_back(e);
    c->order_set.push_back(0);
  }
  if (hipEventRecord(c->order_ev[slot], c->stream) != hipSuccess) return BG_E_HIP;
  c->order_set[slot] = 1;
  return 0;
}

extern "C" int bg_copy_fence(bg_ctx* c, int slot) {
  if (!c || slot < 0) return BG_E_ARG;
  hipEvent_t ev = nullptr;
  {
    std::lock_guard<std::mutex> g(c->copy_mu);
    if (slot >= (int)c->copy_ev.size()) return BG_E_ARG;
    ev = c->copy_ev[slot];
  }
  BG_HIP(c, hipStreamWaitEvent(c->stream, ev, 0));
  return 0;
}

extern "C" void bg_file_image_close(bg_file_image* m) {
  if (!m) return;
  if (m->registered) (void)hipHostUnregister((void*)m->data);
  if (m->data) {
    std::lock_guard<std::mutex> g(img_mu);
    auto it = img_fd.find(m->data);
    if (it != img_fd.end()) {
      close(it->second);
      img_fd.erase(it);
    }
  }
  if (m->data && m->n) munmap((void*)m->data, (size_t)m->n);
  memset(m, 0, sizeof(*m));
}

// a regular file straight into a new device buffer (the four calls above, in order); the
// host image is released once the copy completed
extern "C" int bg_read_file_device(bg_ctx* c, const char* path, void** out, uint64_t* nbytes) {
  if (!c || !path || !out || !nbytes) return BG_E_ARG;
  *out = nullptr;
  *nbytes = 0;
  bg_file_image m;
  int rc = bg_file_image_open(path, &m);
  if (rc) return bg_fail(c, rc, std::string("cannot read ") + path);
  const uint64_t n = m.n;
  bg_bind(c);
  (void)bg_file_image_register(&m);
  void* d = nullptr;
  rc = bg_file_image_to_device(c, &m, 0, n, &d);
  if (!rc) rc = bg_hip_ok(c, hipStreamSynchronize(c->stream));
  bg_file_image_close(&m);
  if (rc) {
    bg_release(c, d);
    return rc;
  }
  bg_mark(c, "read");
  *out = d;
  *nbytes = n;
  return 0;
}

// Output to a regular file: BG_WR_THREADS threads each stage ring-slot chunks (D2H by DMA on
// ctx's stream) and pwrite(2) them at their offsets, so the page-cache copies of several
// chunks run at once. Measured on the box (tools/out_probe.cpp, 0.92 GB): one write(2)
// stream 88-165 ms, pwrite from 4 threads ~105 ms, a shared mapping of the file filled by DMA
// 128 ms (page allocation through faults does not scale with threads: 285 ms with 4).
// Anything else (pipes, terminals, appends): the same chunks written in order by one thread.
// (at >= 0: pwrite(2) at that offset and leave the file position alone: bg_pwrite_device)
#define BG_WR_THREADS 4
static int write_device_ring(bg_ctx* c, const void* d, uint64_t n, int fd, off_t at = -1) {
  if (at < 0 && c->out_skip) {  // bg_set_output_skip: this much of the stream is out already
    const uint64_t k = std::min(c->out_skip, n);
    c->out_skip -= k;
    d = (const char*)d + k;
    n -= k;
    if (n == 0) return 0;
  }
  int rc = ring_get(c);
  if (rc) return rc;
  struct stat st;
  const int fl = fcntl(fd, F_GETFL);
  const off_t off0 = at >= 0 ? at : lseek(fd, 0, SEEK_CUR);
  const char* par = getenv("BEDGPU_WRITE_PAR");  // 0: one thread, write(2)
  const bool pw = at >= 0 || (fstat(fd, &st) == 0 && S_ISREG(st.st_mode) && fl >= 0 && !(fl & O_APPEND) &&
                              off0 >= 0 && !(par && strcmp(par, "0") == 0));
  const uint64_t CH = BG_RING_CH, nch = (n + CH - 1) / CH;
  const int T = pw ? (int)std::min<uint64_t>(BG_WR_THREADS, nch) : 1;
  const int per = BG_RING_SLOTS / BG_WR_THREADS;
  std::mutex mu;
  std::atomic<int> bad{0};
  // one writer: chunks in order, the DMA of the next `per` chunks queued ahead of write(2)
  auto issue = [&](uint64_t k, int sl) -> bool {
    const uint64_t o = k * CH, len = std::min(CH, n - o);
    std::lock_guard<std::mutex> g(mu);
    return hipMemcpyAsync(c->ring[sl], (const char*)d + o, len, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
           hipEventRecord(c->ring_ev[sl], c->stream) == hipSuccess;
  };
  auto worker = [&](int t) {
    if (hipSetDevice(c->device) != hipSuccess) { bad = 1; return; }
    std::vector<uint64_t> mine;
    for (uint64_t k = (uint64_t)t; k < nch; k += (uint64_t)T) mine.push_back(k);
    const size_t depth = std::min<size_t>(per, mine.size());
    for (size_t q = 0; q < depth; ++q)
      if (!issue(mine[q], t * per + (int)(q % per))) { bad = 1; return; }
    for (size_t q = 0; q < mine.size() && !bad; ++q) {
      const int sl = t * per + (int)(q % per);
      const uint64_t k = mine[q], o = k * CH, len = std::min(CH, n - o);
      if (hipEventSynchronize(c->ring_ev[sl]) != hipSuccess) { bad = 1; return; }
      uint64_t w = 0;
      while (w < len) {
        const ssize_t r = pw ? pwrite(fd, c->ring[sl] + w, len - w, off0 + (off_t)(o + w))
                             : write(fd, c->ring[sl] + w, len - w);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) { bad = 2; return; }
        w += (uint64_t)r;
      }
      if (q + depth < mine.size() && !issue(mine[q + depth], sl)) { bad = 1; return; }
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t) th.emplace_back(worker, t);
  worker(0);
  for (auto& x : th) x.join();
  hipStreamSynchronize(c->stream);
  if (bad == 2) return bg_fail(c, BG_E_IO, std::string("write failed: ") + strerror(errno));
  if (bad) return bg_fail(c, BG_E_HIP, "bg_write_device copy");
  if (pw && at < 0 && lseek(fd, off0 + (off_t)n, SEEK_SET) < 0)
    return bg_fail(c, BG_E_IO, std::string("seek failed: ") + strerror(errno));
  return 0;
}

extern "C" int bg_set_output_skip(bg_ctx* c, uint64_t n) {
  if (!c) return BG_E_ARG;
  c->out_skip = n;
  return 0;
}

extern "C" int bg_output_skip_left(const bg_ctx* c, uint64_t* n) {
  if (!c || !n) return BG_E_ARG;
  *n = c->out_skip;
  return 0;
}

// n bytes of device memory to the regular file fd at offset `at` (pwrite: the file position
// is not used or moved), so several devices can write their parts of one output at once
extern "C" int bg_pwrite_device(bg_ctx* c, const void* d, uint64_t n, int fd, int64_t at) {
  if (!c || (!d && n) || at < 0) return BG_E_ARG;
  if (n == 0) return 0;
  bg_bind(c);
  return write_device_ring(c, d, n, fd, (off_t)at);
}

// streams n bytes of device memory to fd (write_device_ring)
extern "C" int bg_write_device(bg_ctx* c, const void* d, uint64_t n, int fd) {
  if (!c || (!d && n)) return BG_E_ARG;
  if (n == 0) return 0;
  bg_bind(c);
  const int rc = write_device_ring(c, d, n, fd);
  bg_mark(c, "write");
  return rc;
}

// formats on the device, then streams the text to fd
extern "C" int bg_result_write(bg_ctx* c, bg_result* r, int fd) {
  uint64_t n = 0;
  int rc = bg_result_format(c, r, &n);
  if (rc && rc != BG_E_VISITOR) return rc;
  const int wr = bg_write_device(c, r->text, n, fd);
  return wr ? wr : rc;  // BG_E_VISITOR after the text before the stop is written
}

// host parts (pinned, registered or pageable) copied back to back into one new device
// buffer: a chromosome shard of a file assembled on the GPU that will parse it
extern "C" int bg_device_gather_host(bg_ctx* c, int n, const void* const* parts, const uint64_t* lens,
                                     void** out, uint64_t* total) {
  if (!c || n < 0 || !out || !total || (n && (!parts || !lens))) return BG_E_ARG;
  bg_bind(c);
  uint64_t t = 0;
  for (int k = 0; k < n; ++k) t += lens[k];
  char* d = (char*)bg_alloc(c, t + 64);
  if (!d) return BG_E_NOMEM;
  uint64_t o = 0;
  for (int k = 0; k < n; ++k) {  // through the staging ring (pageable or registered parts alike)
    const int rc = ring_h2d(c, d + o, (const char*)parts[k], lens[k]);
    if (rc) {
      hipStreamSynchronize(c->stream);
      bg_release(c, d);
      return rc;
    }
    o += lens[k];
  }
  *out = d;
  *total = t;
  return 0;
}

// ---------------------------------------------------------------------------------------
// Output queue (bg_writer): device texts handed over in order are copied D2H on a stream of
// the queue's own into the ring's writer slots and written with write(2) by one host thread,
// so the output of one chromosome group goes out while the next group is read (H2D on ctx's
// stream, the other direction of the link) and computed. One writer thread: buffered writes
// to one file serialise on its inode lock anyway (tools/out_probe.cpp measurements above).
// ---------------------------------------------------------------------------------------
struct bg_writer {
  bg_ctx* c = nullptr;
  int fd = -1;
  hipStream_t st = nullptr;
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  struct Job {
    const char* d;
    uint64_t n;
    hipEvent_t ready;
  };
  std::deque<Job> q;
  std::vector<hipEvent_t> spare;  // ready events the writer has finished with
  uint64_t done = 0;
  bool closing = false;
  int err = 0;  // BG_E_IO / BG_E_HIP
  int eno = 0;
};

static void writer_loop(bg_writer* w) {
  bg_ctx* c = w->c;
  if (hipSetDevice(c->device) != hipSuccess ||
      hipStreamCreateWithFlags(&w->st, hipStreamNonBlocking) != hipSuccess) {
    std::lock_guard<std::mutex> g(w->mu);
    w->err = BG_E_HIP;
  }
  const uint64_t CH = BG_RING_CH;
  for (;;) {
    bg_writer::Job J;
    {
      std::unique_lock<std::mutex> g(w->mu);
      w->cv.wait(g, [&] { return w->closing || !w->q.empty(); });
      if (w->q.empty()) return;  // closing, everything written
      J = w->q.front();
    }
    int bad = 0, eno = 0;
    {
      std::lock_guard<std::mutex> g(w->mu);
      bad = w->err;
    }
    if (!bad && J.n) {
      const uint64_t nch = (J.n + CH - 1) / CH;
      auto slot = [&](uint64_t k) { return BG_RING_SLOTS + (int)(k % BG_WR_SLOTS); };
      auto issue = [&](uint64_t k) -> bool {
        const uint64_t o = k * CH, len = std::min(CH, J.n - o);
        const int sl = slot(k);
        return hipMemcpyAsync(c->ring[sl], J.d + o, len, hipMemcpyDeviceToHost, w->st) == hipSuccess &&
               hipEventRecord(c->ring_ev[sl], w->st) == hipSuccess;
      };
      if (hipStreamWaitEvent(w->st, J.ready, 0) != hipSuccess) bad = BG_E_HIP;
      const uint64_t depth = std::min<uint64_t>(BG_WR_SLOTS, nch);
      for (uint64_t k = 0; k < depth && !bad; ++k)
        if (!issue(k)) bad = BG_E_HIP;
      for (uint64_t k = 0; k < nch && !bad; ++k) {
        const int sl = slot(k);
        if (hipEventSynchronize(c->ring_ev[sl]) != hipSuccess) { bad = BG_E_HIP; break; }
        const uint64_t o = k * CH, len = std::min(CH, J.n - o);
        uint64_t x = 0;
        while (x < len) {
          const ssize_t r = write(w->fd, c->ring[sl] + x, len - x);
          if (r < 0 && errno == EINTR) continue;
          if (r <= 0) { bad = BG_E_IO; eno = r < 0 ? errno : EIO; break; }
          x += (uint64_t)r;
        }
        if (!bad && k + depth < nch && !issue(k + depth)) bad = BG_E_HIP;
      }
      if (bad) (void)hipStreamSynchronize(w->st);  // no copy into a slot stays in flight
    }
    std::lock_guard<std::mutex> g(w->mu);
    if (bad && !w->err) { w->err = bad; w->eno = eno; }
    w->spare.push_back(J.ready);
    w->q.pop_front();
    ++w->done;
    w->cv.notify_all();
  }
}

extern "C" int bg_writer_open(bg_ctx* c, int fd, bg_writer** out) {
  if (!c || !out || fd < 0) return BG_E_ARG;
  *out = nullptr;
  bg_bind(c);
  int rc = ring_get(c);  // the writer slots are pinned with the ring
  if (rc) return rc;
  bg_writer* w = new bg_writer();
  w->c = c;
  w->fd = fd;
  w->th = std::thread(writer_loop, w);
  *out = w;
  return 0;
}

extern "C" int bg_writer_push(bg_writer* w, const void* d, uint64_t n) {
  if (!w || (!d && n)) return BG_E_ARG;
  bg_ctx* c = w->c;
  hipEvent_t ev = nullptr;
  {
    std::lock_guard<std::mutex> g(w->mu);
    if (w->err) return bg_fail(c, w->err, "output queue failed");
    if (!w->spare.empty()) { ev = w->spare.back(); w->spare.pop_back(); }
  }
  if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess)
    return bg_fail(c, BG_E_HIP, "output queue event");
  BG_HIP(c, hipEventRecord(ev, c->stream));  // the text is complete once ctx's stream gets here
  std::lock_guard<std::mutex> g(w->mu);
  w->q.push_back({(const char*)d, n, ev});
  w->cv.notify_all();
  return 0;
}

extern "C" uint64_t bg_writer_done(bg_writer* w) {
  if (!w) return 0;
  std::lock_guard<std::mutex> g(w->mu);
  return w->done;
}

extern "C" int bg_writer_close(bg_writer* w) {
  if (!w) return BG_E_ARG;
  {
    std::lock_guard<std::mutex> g(w->mu);
    w->closing = true;
    w->cv.notify_all();
  }
  w->th.join();
  bg_ctx* c = w->c;
  int rc = w->err;
  if (rc == BG_E_IO) bg_fail(c, rc, std::string("write failed: ") + strerror(w->eno));
  else if (rc) bg_fail(c, rc, "output queue copy failed");
  for (auto e : w->spare) hipEventDestroy(e);
  if (w->st) hipStreamDestroy(w->st);
  delete w;
  return rc;
}

extern "C" int bg_bind(bg_ctx* c) {
  if (!c) return BG_E_ARG;
  int d = -1;
  if (hipGetDevice(&d) != hipSuccess || d != c->device) BG_HIP(c, hipSetDevice(c->device));
  return 0;
}

extern "C" void* bg_host_alloc(uint64_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return nullptr;
  return p;
}

extern "C" void bg_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

extern "C" void bg_result_free(bg_result* r) {
  if (!r) return;
  bg_ctx* c = r->ctx;
  bg_release(c, r->s);
  bg_release(c, r->e);
  bg_release(c, r->seg_off);
  bg_release(c, r->seg_boff);
  bg_release(c, r->tbytes);
  bg_release(c, r->rows);
  bg_release(c, r->rlen);
  bg_release(c, r->cnt);
  bg_release(c, r->isum);
  bg_release(c, r->vmin);
  bg_release(c, r->vmax);
  bg_release(c, r->bases);
  bg_release(c, r->uniq);
  bg_release(c, r->isq);
  bg_release(c, r->dsum);
  bg_release(c, r->dsq);
  for (int q = 0; q < 16; ++q) bg_release(c, r->tmv[q]);
  bg_release(c, r->rrank);
  bg_release(c, r->wlo);
  bg_release(c, r->whi);
  bg_release(c, (void*)r->lrows.idx);
  bg_release(c, (void*)r->lrows.ls);
  bg_release(c, (void*)r->lrows.coff);
  bg_release(c, r->zin);
  bg_release(c, r->zout);
  bg_release(c, r->maddr);
  bg_release(c, r->left);
  bg_release(c, r->right);
  bg_release(c, r->text);
  bg_release(c, r->toff);
  if (r->own_set) bg_set_free(r->set);
  delete r;
}

// e2e_probe — measures the host-side costs of getting a page-cached BED file into HBM on the
// box (round-3 ingest design): HIP init pieces, pread into a pinned ring (the current
// bg_read_file_device), hipHostRegister of the file's own mmap (DMA straight from the page
// cache), and a plain anonymous buffer filled by threads then registered.
// usage: e2e_probe <file> [threads]
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

using clk = std::chrono::steady_clock;
static double ms(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); }
#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

__global__ void k_touch(const unsigned char* p, uint64_t n, unsigned long long* out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long s = 0;
  for (; i < n; i += (uint64_t)gridDim.x * blockDim.x * 4096) s += p[i];
  if (s == 12345) *out = s;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const int T = argc > 2 ? atoi(argv[2]) : 8;
  auto t0 = clk::now();
  CK(hipInit(0));
  auto t1 = clk::now();
  CK(hipSetDevice(0));
  auto t2 = clk::now();
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto t3 = clk::now();
  unsigned long long* dout;
  CK(hipMalloc(&dout, 8));
  k_touch<<<1, 64, 0, s>>>((const unsigned char*)dout, 8, dout);
  CK(hipStreamSynchronize(s));
  auto t4 = clk::now();
  printf("init: hipInit %.1f ms, hipSetDevice %.1f ms, stream %.1f ms, first kernel %.1f ms\n", ms(t0, t1),
         ms(t1, t2), ms(t2, t3), ms(t3, t4));

  int fd = open(argv[1], O_RDONLY);
  struct stat st;
  fstat(fd, &st);
  const uint64_t n = (uint64_t)st.st_size;
  char* d;
  auto a0 = clk::now();
  CK(hipMalloc(&d, n + 64));
  auto a1 = clk::now();
  CK(hipMemsetAsync(d, 0, n, s));
  CK(hipStreamSynchronize(s));
  auto a2 = clk::now();
  printf("hipMalloc %.2f GB %.1f ms, first memset %.1f ms\n", n / 1e9, ms(a0, a1), ms(a1, a2));

  // (1) mmap + hipHostRegister of the whole file, one copy
  for (int flags : {hipHostRegisterReadOnly, hipHostRegisterDefault}) {
    auto b0 = clk::now();
    char* m = (char*)mmap(nullptr, n, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, 0);
    auto b1 = clk::now();
    hipError_t e = hipHostRegister(m, n, flags);
    auto b2 = clk::now();
    if (e != hipSuccess) {
      printf("register(flags %d) of the file mmap failed: %s (mmap %.1f ms, %.1f ms)\n", flags,
             hipGetErrorString(e), ms(b0, b1), ms(b1, b2));
      (void)hipGetLastError();
      munmap(m, n);
      continue;
    }
    CK(hipMemcpyAsync(d, m, n, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    auto b3 = clk::now();
    CK(hipHostUnregister(m));
    auto b4 = clk::now();
    munmap(m, n);
    printf("file mmap+register(flags %d): mmap %.1f ms, register %.1f ms, copy %.1f ms (%.1f GB/s), unregister %.1f ms\n",
           flags, ms(b0, b1), ms(b1, b2), ms(b2, b3), n / 1e6 / ms(b2, b3), ms(b3, b4));
  }

  // (2) chunked: T threads each register 64 MiB pieces of the file mmap and copy them
  {
    const uint64_t CH = 64ull << 20;
    auto b0 = clk::now();
    char* m = (char*)mmap(nullptr, n, PROT_READ, MAP_SHARED, fd, 0);
    const uint64_t nch = (n + CH - 1) / CH;
    std::atomic<int> bad{0};
    std::vector<std::thread> th;
    std::vector<hipStream_t> ss(T);
    for (auto& x : ss) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    auto b1 = clk::now();
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t]() {
        (void)hipSetDevice(0);
        for (uint64_t k = t; k < nch; k += T) {
          const uint64_t off = k * CH, len = std::min(CH, n - off);
          if (hipHostRegister(m + off, len, hipHostRegisterReadOnly) != hipSuccess) { bad = 1; return; }
          if (hipMemcpyAsync(d + off, m + off, len, hipMemcpyHostToDevice, ss[t]) != hipSuccess) { bad = 1; return; }
          (void)hipStreamSynchronize(ss[t]);
          (void)hipHostUnregister(m + off);
        }
      });
    for (auto& x : th) x.join();
    auto b2 = clk::now();
    munmap(m, n);
    printf("chunked register+copy, %d threads: setup %.1f ms, total %.1f ms (%.1f GB/s)%s\n", T, ms(b0, b1),
           ms(b1, b2), n / 1e6 / ms(b1, b2), bad ? " FAILED" : "");
  }

  // (3) pread into a pinned ring (the current reader), T threads x 2 slots of 2 MiB
  {
    const uint64_t CH = 2ull << 20;
    std::vector<char*> slot(2 * T);
    auto b0 = clk::now();
    for (auto& p : slot) CK(hipHostMalloc((void**)&p, CH, hipHostMallocDefault));
    std::vector<hipStream_t> ss(2);
    for (auto& x : ss) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    std::vector<hipEvent_t> ev(2 * T);
    for (auto& x : ev) CK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
    auto b1 = clk::now();
    const uint64_t nch = (n + CH - 1) / CH;
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t]() {
        (void)hipSetDevice(0);
        uint64_t j = 0;
        for (uint64_t k = t; k < nch; k += T, ++j) {
          const int sl = 2 * t + (int)(j & 1);
          (void)hipEventSynchronize(ev[sl]);
          const uint64_t off = k * CH, len = std::min(CH, n - off);
          uint64_t got = 0;
          while (got < len) {
            ssize_t r = pread(fd, slot[sl] + got, len - got, off + got);
            if (r <= 0) break;
            got += r;
          }
          (void)hipMemcpyAsync(d + off, slot[sl], len, hipMemcpyHostToDevice, ss[t % 2]);
          (void)hipEventRecord(ev[sl], ss[t % 2]);
        }
      });
    for (auto& x : th) x.join();
    for (auto& x : ss) (void)hipStreamSynchronize(x);
    auto b2 = clk::now();
    printf("pinned ring pread, %d threads: setup %.1f ms, total %.1f ms (%.1f GB/s)\n", T, ms(b0, b1), ms(b1, b2),
           n / 1e6 / ms(b1, b2));
  }

  // (4) plain pread into anonymous memory by T threads (what could run during HIP init),
  //     then register it and copy
  {
    auto b0 = clk::now();
    char* m = (char*)mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    madvise(m, n, MADV_HUGEPAGE);
    const uint64_t CH = 8ull << 20;
    const uint64_t nch = (n + CH - 1) / CH;
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t]() {
        for (uint64_t k = t; k < nch; k += T) {
          const uint64_t off = k * CH, len = std::min(CH, n - off);
          uint64_t got = 0;
          while (got < len) {
            ssize_t r = pread(fd, m + off + got, len - got, off + got);
            if (r <= 0) break;
            got += r;
          }
        }
      });
    for (auto& x : th) x.join();
    auto b1 = clk::now();
    hipError_t e = hipHostRegister(m, n, hipHostRegisterDefault);
    auto b2 = clk::now();
    if (e == hipSuccess) {
      CK(hipMemcpyAsync(d, m, n, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
    }
    auto b3 = clk::now();
    printf("anon pread %d threads %.1f ms (%.1f GB/s); register %.1f ms%s; copy %.1f ms\n", T, ms(b0, b1),
           n / 1e6 / ms(b0, b1), ms(b1, b2), e == hipSuccess ? "" : " FAILED", ms(b2, b3));
    auto b4 = clk::now();
    if (e == hipSuccess) (void)hipHostUnregister(m);
    munmap(m, n);
    printf("  unregister+munmap %.1f ms\n", ms(b3, clk::now()) - ms(b3, b4) + ms(b4, clk::now()));
  }
  // (5) hipMemcpy straight from a pageable mapping of the file (runtime staging)
  {
    char* m = (char*)mmap(nullptr, n, PROT_READ, MAP_SHARED, fd, 0);
    auto b0 = clk::now();
    CK(hipMemcpy(d, m, n, hipMemcpyHostToDevice));
    auto b1 = clk::now();
    munmap(m, n);
    printf("pageable hipMemcpy from the file mmap: %.1f ms (%.1f GB/s)\n", ms(b0, b1), n / 1e6 / ms(b0, b1));
  }
  auto z0 = clk::now();
  CK(hipFree(d));
  printf("hipFree %.1f ms\n", ms(z0, clk::now()));
  return 0;
}

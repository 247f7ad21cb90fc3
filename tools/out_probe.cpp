// out_probe — ways to land N bytes of HBM text in an output file on the box (round-3 e2e):
// write(2) of a registered bounce buffer, pwrite from several threads, a shared mapping of the
// file populated by k threads (or by the registration) and filled by DMA.
// usage: out_probe <dir> [MB]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <string>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif
using clk = std::chrono::steady_clock;
static double ms(clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); }

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  const uint64_t n = (uint64_t)(argc > 2 ? atoi(argv[2]) : 918) << 20;
  (void)hipSetDevice(0);
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  char* d = nullptr;
  (void)hipMalloc(&d, n);
  (void)hipMemsetAsync(d, 'x', n, s);
  (void)hipStreamSynchronize(s);
  const uint64_t CH = 64ull << 20;
  auto path = [&](const char* t) { return dir + "/out_probe_" + t; };
  {  // (a) registered bounce buffers + write(2)
    const std::string p = path("a");
    auto t0 = clk::now();
    int fd = open(p.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    char* b = (char*)malloc(2 * CH);
    (void)hipHostRegister(b, 2 * CH, 0);
    for (uint64_t o = 0, k = 0; o < n; o += CH, ++k) {
      const uint64_t l = std::min(CH, n - o);
      (void)hipMemcpyAsync(b + (k % 2) * CH, d + o, l, hipMemcpyDeviceToHost, s);
      (void)hipStreamSynchronize(s);
      if (write(fd, b + (k % 2) * CH, l) != (ssize_t)l) return 1;
    }
    close(fd);
    printf("(a) write(2), 64 MiB chunks: %.1f ms\n", ms(t0));
    (void)hipHostUnregister(b);
    free(b);
    unlink(p.c_str());
  }
  for (int T : {1, 4, 8}) {  // (b) pwrite from T threads (each its own bounce buffer)
    const std::string p = path("b");
    auto t0 = clk::now();
    int fd = open(p.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t]() {
        char* b = (char*)malloc(CH);
        (void)hipHostRegister(b, CH, 0);
        hipStream_t ls = s;
        for (uint64_t o = (uint64_t)t * CH; o < n; o += (uint64_t)T * CH) {
          const uint64_t l = std::min(CH, n - o);
          (void)hipMemcpyAsync(b, d + o, l, hipMemcpyDeviceToHost, ls);
          (void)hipStreamSynchronize(ls);
          if (pwrite(fd, b, l, o) != (ssize_t)l) abort();
        }
        (void)hipHostUnregister(b);
        free(b);
      });
    for (auto& x : th) x.join();
    close(fd);
    printf("(b) pwrite from %d threads: %.1f ms\n", T, ms(t0));
    unlink(p.c_str());
  }
  for (int T : {0, 1, 4}) {  // (c) mapping populated by T threads (0: by the registration), DMA
    const std::string p = path("c");
    auto t0 = clk::now();
    int fd = open(p.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0644);
    if (ftruncate(fd, n)) return 1;
    char* m = (char*)mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    auto t1 = clk::now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t]() {
        const uint64_t per = ((n / T) + 4095) & ~4095ull, a = t * per;
        if (a < n) madvise(m + a, std::min(per, n - a), MADV_POPULATE_WRITE);
      });
    for (auto& x : th) x.join();
    const double tp = ms(t1);
    auto t2 = clk::now();
    const hipError_t e = hipHostRegister(m, n, 0);
    const double tr = ms(t2);
    auto t3 = clk::now();
    (void)hipMemcpyAsync(m, d, n, hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    const double tc = ms(t3);
    (void)hipHostUnregister(m);
    munmap(m, n);
    close(fd);
    printf("(c) mmap, populate by %d threads %.1f ms, register %.1f ms (%s), DMA %.1f ms: total %.1f ms\n", T, tp,
           tr, e == hipSuccess ? "ok" : "FAILED", tc, ms(t0));
    unlink(p.c_str());
  }
  {  // (d) pageable D2H into a malloc'd buffer, then write(2) (runtime staging)
    const std::string p = path("d");
    auto t0 = clk::now();
    int fd = open(p.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    char* b = (char*)malloc(n);
    (void)hipMemcpy(b, d, n, hipMemcpyDeviceToHost);
    const double tc = ms(t0);
    if (write(fd, b, n) != (ssize_t)n) return 1;
    close(fd);
    printf("(d) pageable D2H %.1f ms + one write(2): total %.1f ms\n", tc, ms(t0));
    free(b);
    unlink(p.c_str());
  }
  return 0;
}

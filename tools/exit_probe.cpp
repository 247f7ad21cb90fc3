// exit_probe — process start / exit costs of a HIP process on the box (round-3 e2e work).
// Prints CLOCK_MONOTONIC at main entry and right before exit so the caller can split its
// wall clock into (spawn + loader), work, and (teardown).
// usage: exit_probe none | init | alloc <GB> [free] [full] | pin <MB> [full] | reg <file> [full]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <vector>

static double now() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

int main(int argc, char** argv) {
  const double t0 = now();
  printf("main %.6f\n", t0);
  const char* mode = argc > 1 ? argv[1] : "none";
  bool full = false, dofree = false;
  for (int i = 2; i < argc; ++i) {
    if (!strcmp(argv[i], "full")) full = true;
    if (!strcmp(argv[i], "free")) dofree = true;
  }
  std::vector<void*> bufs;
  if (!strcmp(mode, "streams")) {  // streams <n>: hipSetDevice, then n streams each running a kernel
    const int n = atoi(argv[2]);
    (void)hipSetDevice(0);
    const double a = now();
    void* d = nullptr;
    (void)hipMalloc(&d, 64);
    (void)hipMemsetAsync(d, 0, 64, 0);  // the null stream
    (void)hipDeviceSynchronize();
    const double b = now();
    std::vector<hipStream_t> ss(n);
    for (auto& x : ss) (void)hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
    const double c = now();
    for (auto& x : ss) (void)hipMemsetAsync(d, 1, 64, x);
    (void)hipDeviceSynchronize();
    const double e = now();
    printf("setdevice %.1f ms, null-stream first op %.1f ms, %d streams create %.1f ms, first op %.1f ms\n",
           1e3 * (a - t0), 1e3 * (b - a), n, 1e3 * (c - b), 1e3 * (e - c));
  } else if (strcmp(mode, "none") != 0) {
    hipStream_t s;
    (void)hipSetDevice(0);
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    printf("init %.1f ms\n", 1e3 * (now() - t0));
    if (!strcmp(mode, "alloc")) {
      const double gb = atof(argv[2]);
      const size_t each = 1ull << 30;
      for (double g = 0; g < gb; g += 1.0) {
        void* p = nullptr;
        if (hipMalloc(&p, each) != hipSuccess) break;
        (void)hipMemsetAsync(p, 1, each, s);
        bufs.push_back(p);
      }
      (void)hipStreamSynchronize(s);
      printf("alloc+memset %zu GB done %.1f ms\n", bufs.size(), 1e3 * (now() - t0));
      if (dofree) {
        const double f0 = now();
        for (void* p : bufs) (void)hipFree(p);
        printf("hipFree %.1f ms\n", 1e3 * (now() - f0));
      }
    } else if (!strcmp(mode, "pin")) {
      const size_t mb = (size_t)atoi(argv[2]);
      for (size_t k = 0; k < mb / 2; ++k) {
        void* p = nullptr;
        (void)hipHostMalloc(&p, 2u << 20, hipHostMallocDefault);
      }
      printf("pinned %zu MB done %.1f ms\n", mb, 1e3 * (now() - t0));
    } else if (!strcmp(mode, "reg")) {
      int fd = open(argv[2], O_RDONLY);
      struct stat st;
      fstat(fd, &st);
      char* m = (char*)mmap(nullptr, st.st_size, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, 0);
      (void)hipHostRegister(m, st.st_size, hipHostRegisterDefault);
      void* d = nullptr;
      (void)hipMalloc(&d, st.st_size);
      (void)hipMemcpyAsync(d, m, st.st_size, hipMemcpyHostToDevice, s);
      (void)hipStreamSynchronize(s);
      printf("registered + copied %.2f GB done %.1f ms\n", st.st_size / 1e9, 1e3 * (now() - t0));
    }
  }
  const double t1 = now();
  printf("exit %.6f\n", t1);
  fflush(stdout);
  if (full) return 0;
  _exit(0);
}

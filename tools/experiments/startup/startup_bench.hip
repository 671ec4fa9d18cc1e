// Start-up cost of the HIP runtime pieces the application needs before its
// first template (round 3, whole-process wall time on the reference protocol):
// runtime init, stream (HW queue) creation, first copy / first kernel per
// stream, sequential vs from one thread per stream.
// usage: startup_bench <seq|par> [streams] [teardown: none|free|all] [MB per stream]
// prints the wall-clock time (epoch ms) just before _exit so that the caller
// can time the process exit (GPU teardown by the kernel driver)
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

using clk = std::chrono::steady_clock;
static double ms_since(clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); }

__global__ void touch(float* p) { p[threadIdx.x] += 1.0f; }

static int g_mb = 72;

struct Pipe {
  hipStream_t s = nullptr;
  float* d = nullptr;
  double t_create = 0, t_copy = 0, t_kernel = 0, t_alloc = 0;
};

static void bring_up(Pipe& p, const float* host) {
  auto t = clk::now();
  (void)hipStreamCreateWithFlags(&p.s, hipStreamNonBlocking);
  p.t_create = ms_since(t);
  t = clk::now();
  (void)hipMalloc(&p.d, static_cast<size_t>(g_mb) << 20);
  p.t_alloc = ms_since(t);
  t = clk::now();
  (void)hipMemcpyAsync(p.d, host, 1 << 20, hipMemcpyHostToDevice, p.s);
  (void)hipStreamSynchronize(p.s);
  p.t_copy = ms_since(t);
  t = clk::now();
  hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, p.s, p.d);
  (void)hipStreamSynchronize(p.s);
  p.t_kernel = ms_since(t);
}

int main(int argc, char** argv) {
  const auto t0 = clk::now();
  const bool par = argc > 1 && std::strcmp(argv[1], "par") == 0;
  const int n = argc > 2 ? std::atoi(argv[2]) : 3;
  const char* teardown = argc > 3 ? argv[3] : "none";
  if (argc > 4) g_mb = std::atoi(argv[4]);
  int ndev = 0;
  (void)hipGetDeviceCount(&ndev);
  const double t_init = ms_since(t0);
  auto t = clk::now();
  (void)hipSetDevice(0);
  (void)hipFree(nullptr);
  const double t_ctx = ms_since(t);
  std::vector<float> host(1 << 18, 1.0f);
  std::vector<Pipe> pipes(n);
  t = clk::now();
  if (par) {
    std::vector<std::thread> th;
    for (int i = 0; i < n; ++i) th.emplace_back([&, i] { (void)hipSetDevice(0); bring_up(pipes[i], host.data()); });
    for (auto& x : th) x.join();
  } else {
    for (int i = 0; i < n; ++i) bring_up(pipes[i], host.data());
  }
  const double t_pipes = ms_since(t);
  t = clk::now();
  float* d0 = nullptr;
  (void)hipMalloc(&d0, 1 << 20);
  (void)hipMemcpy(d0, host.data(), 1 << 20, hipMemcpyHostToDevice);  // null stream
  const double t_null = ms_since(t);
  printf("{\"mode\": \"%s\", \"streams\": %d, \"devices\": %d, \"init_ms\": %.2f, \"ctx_ms\": %.2f, \"pipes_ms\": %.2f, "
         "\"null_stream_copy_ms\": %.2f, \"per_stream\": [",
         par ? "par" : "seq", n, ndev, t_init, t_ctx, t_pipes, t_null);
  for (int i = 0; i < n; ++i)
    printf("%s{\"create\": %.2f, \"alloc72MB\": %.2f, \"first_copy\": %.2f, \"first_kernel\": %.2f}", i ? ", " : "",
           pipes[i].t_create, pipes[i].t_alloc, pipes[i].t_copy, pipes[i].t_kernel);
  printf("], \"total_ms\": %.2f", ms_since(t0));
  t = clk::now();
  if (std::strcmp(teardown, "none") != 0) {
    for (auto& p : pipes) (void)hipFree(p.d);
    (void)hipFree(d0);
    if (std::strcmp(teardown, "all") == 0)
      for (auto& p : pipes) (void)hipStreamDestroy(p.s);
  }
  const double t_td = ms_since(t);
  const double epoch = std::chrono::duration<double, std::milli>(std::chrono::system_clock::now().time_since_epoch()).count();
  printf(", \"teardown\": \"%s\", \"teardown_ms\": %.2f, \"epoch_ms_before_exit\": %.3f}\n", teardown, t_td, epoch);
  fflush(stdout);
  _exit(0);
}

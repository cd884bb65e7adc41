// hipGraph A/B for the per-scan device chain (VERDICT r03 "measure hipGraph capture"): a chain of
// six dependent kernels shaped like the C2 scan front (k_points 1,024 blocks, k_bins_scale 768, its
// fold 1, k_pt 256, its fold 1, k_tile_order 1), launched
//   stream  -- six hipLaunchKernelGGL calls on one stream, then a stream sync
//   graph   -- the same six captured once into a hipGraph, one hipGraphLaunch per chain
//   graphup -- the graph with the first node's arguments rewritten before every launch
//              (hipGraphExecKernelNodeSetParams: the per-scan pointers / scan times)
// and timed end to end from the host (launch call -> sync returns), median over 2,000 chains.
// Build: hipcc -O3 --offload-arch=gfx950 tools/graph_ab.hip -o tools/graph_ab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

struct Args {
  double* buf;
  int n;
  int iters;
  double s;
};

__global__ __launch_bounds__(256) void k_work(Args a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  double x = a.buf[i];
  for (int k = 0; k < a.iters; ++k) x = fma(x, 0.999999, a.s);
  a.buf[i] = x;
}

using clk = std::chrono::steady_clock;

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 2000;
  const int blocks[6] = {1024, 768, 1, 256, 1, 1};
  const int iters[6] = {400, 600, 2000, 200, 1500, 800};
  double* buf;
  CHK(hipMalloc(&buf, (size_t)1024 * 256 * sizeof(double)));
  CHK(hipMemset(buf, 0, (size_t)1024 * 256 * sizeof(double)));
  hipStream_t s;
  CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto launch_chain = [&](double sc) {
    for (int k = 0; k < 6; ++k) {
      Args a{buf, blocks[k] * 256, iters[k], k == 0 ? sc : 1e-9};
      hipLaunchKernelGGL(k_work, dim3(blocks[k]), dim3(256), 0, s, a);
    }
  };
  auto median = [](std::vector<double>& v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  // device time of the chain alone (events around one chain)
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  for (int w = 0; w < 50; ++w) launch_chain(1e-9);
  CHK(hipStreamSynchronize(s));
  // stream
  std::vector<double> t_stream, t_dev;
  for (int r = 0; r < reps; ++r) {
    auto t0 = clk::now();
    CHK(hipEventRecord(e0, s));
    launch_chain(1e-9 * r);
    CHK(hipEventRecord(e1, s));
    CHK(hipStreamSynchronize(s));
    t_stream.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    t_dev.push_back(ms * 1e3);
  }
  // graph
  hipGraph_t g;
  hipGraphExec_t ge;
  CHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  launch_chain(1e-9);
  CHK(hipStreamEndCapture(s, &g));
  CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  size_t nn = 0;
  CHK(hipGraphGetNodes(g, nullptr, &nn));
  std::vector<hipGraphNode_t> nodes(nn);
  CHK(hipGraphGetNodes(g, nodes.data(), &nn));
  hipGraphNode_t first = nullptr;
  for (auto nd : nodes) {  // the root kernel node (no dependencies)
    size_t nd_deps = 0;
    CHK(hipGraphNodeGetDependencies(nd, nullptr, &nd_deps));
    if (nd_deps == 0) first = nd;
  }
  for (int w = 0; w < 50; ++w) CHK(hipGraphLaunch(ge, s));
  CHK(hipStreamSynchronize(s));
  std::vector<double> t_graph, t_gdev;
  for (int r = 0; r < reps; ++r) {
    auto t0 = clk::now();
    CHK(hipEventRecord(e0, s));
    CHK(hipGraphLaunch(ge, s));
    CHK(hipEventRecord(e1, s));
    CHK(hipStreamSynchronize(s));
    t_graph.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    t_gdev.push_back(ms * 1e3);
  }
  // graph with a per-launch node update
  hipKernelNodeParams kp{};
  CHK(hipGraphKernelNodeGetParams(first, &kp));
  std::vector<double> t_up, t_upcall;
  for (int r = 0; r < reps; ++r) {
    Args a{buf, blocks[0] * 256, iters[0], 1e-9 * r};
    void* pargs[] = {&a};
    kp.kernelParams = pargs;
    auto t0 = clk::now();
    CHK(hipGraphExecKernelNodeSetParams(ge, first, &kp));
    auto t1 = clk::now();
    CHK(hipGraphLaunch(ge, s));
    CHK(hipStreamSynchronize(s));
    t_up.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
    t_upcall.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
  // launch-call cost alone (host time to enqueue, device busy with a long kernel first)
  std::vector<double> c_stream, c_graph;
  for (int r = 0; r < 200; ++r) {
    Args a{buf, 1024 * 256, 200000, 1e-9};
    hipLaunchKernelGGL(k_work, dim3(1024), dim3(256), 0, s, a);
    auto t0 = clk::now();
    launch_chain(1e-9);
    auto t1 = clk::now();
    CHK(hipGraphLaunch(ge, s));
    auto t2 = clk::now();
    CHK(hipStreamSynchronize(s));
    c_stream.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    c_graph.push_back(std::chrono::duration<double, std::micro>(t2 - t1).count());
  }
  printf("{\"reps\": %d, \"nodes\": %zu, \"stream_wall_us\": %.2f, \"stream_dev_us\": %.2f, \"graph_wall_us\": %.2f, "
         "\"graph_dev_us\": %.2f, \"graph_update_wall_us\": %.2f, \"node_update_call_us\": %.2f, "
         "\"stream_enqueue_us\": %.2f, \"graph_enqueue_us\": %.2f}\n",
         reps, nn, median(t_stream), median(t_dev), median(t_graph), median(t_gdev), median(t_up), median(t_upcall),
         median(c_stream), median(c_graph));
  CHK(hipGraphExecDestroy(ge));
  CHK(hipGraphDestroy(g));
  CHK(hipStreamDestroy(s));
  CHK(hipFree(buf));
  return 0;
}

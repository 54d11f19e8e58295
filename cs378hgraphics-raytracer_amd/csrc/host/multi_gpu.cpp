// multi_gpu.cpp — `ray --gpus N`: one frame tile-sharded over N GPUs of one
// node, one process per GPU, shards gathered over RCCL (SURVEY 8(e);
// the reference's parallel pixel loop, RayTracer.cpp:283-314, split across
// devices instead of threads).
//
//   parent  : parses the scene once (host only, no HIP call), forks N ranks,
//             reaps them as they end; on the first failing rank it ends the
//             others (SIGTERM, then SIGKILL) and returns that rank's status.
//   rank r  : device r; rtx_scene_create; ncclCommInitRank over a unique id
//             that rank 0 publishes in a shared page; renders the 16x16 tiles
//             the deal gives shard r (rtx_render, packed tile order, output
//             left in HBM); ncclGather of the packed RGB8 shards to rank 0.
//   rank 0  : rtx_unpack_tiles of every shard into the frame, writeImage.
//
// The children never exec: each is a fresh process that touches the GPU
// for the first time after the fork (the parent never initialises HIP).
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "cli_opts.h"
#include "rtx.h"
#include "rtx_host.h"

namespace {

// the page the ranks share (created before the fork)
struct Rendezvous {
  std::atomic<int> id_ready;  // 1: uid holds rank 0's ncclUniqueId; -1: rank 0 failed
  std::atomic<int> joined;    // ranks whose scene and buffers are up (ready for the communicator)
  std::atomic<int> failed;    // 1: some rank failed before the collectives
  ncclUniqueId uid;
  double rank_ms[64];         // render + gather wall time per rank
  long long rank_rays[64];
};

// No rank enters ncclCommInitRank (which blocks until all ranks have) until
// every rank got its device, scene and buffers: a rank that fails before
// that publishes it here, and the others return instead of waiting for it
// forever.  (Failures after the collectives started are ended by the
// parent, which terminates the remaining ranks on the first non-zero exit.)
// How long a rank waits for the others (RTX_RANK_WAIT_S seconds, default 600;
// 0: no limit — the parent still ends every rank when one fails).  Each rank
// builds its scene's trees on the CPU before it joins, so a large scene on
// many ranks at once can take a while.
static long rank_wait_s() {
  const char* e = getenv("RTX_RANK_WAIT_S");
  if (e && *e) {
    char* end = nullptr;
    const long v = strtol(e, &end, 10);
    if (end && *end == 0 && v >= 0) return v;
  }
  return 600;
}

static bool waited_too_long(std::chrono::steady_clock::time_point t0) {
  const long lim = rank_wait_s();
  return lim > 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(lim);
}

bool rendezvous_join(Rendezvous* rv, int rank, int nranks) {
  rv->joined.fetch_add(1);
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    if (rv->failed.load()) return false;
    if (rv->joined.load() >= nranks) return true;
    if (waited_too_long(t0)) {
      std::cerr << "rank " << rank << ": the other ranks did not come up" << std::endl;
      rv->failed.store(1);
      return false;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
}

#define NCCL_CHECK(expr, what)                                                      \
  do {                                                                              \
    ncclResult_t r_ = (expr);                                                       \
    if (r_ != ncclSuccess) {                                                        \
      std::cerr << "rank " << rank << ": " << what << ": " << ncclGetErrorString(r_) \
                << std::endl;                                                       \
      return 3;                                                                     \
    }                                                                               \
  } while (0)
#define HIP_CHECK(expr, what)                                                        \
  do {                                                                               \
    hipError_t e_ = (expr);                                                          \
    if (e_ != hipSuccess) {                                                          \
      std::cerr << "rank " << rank << ": " << what << ": " << hipGetErrorString(e_) \
                << std::endl;                                                        \
      return 3;                                                                      \
    }                                                                                \
  } while (0)

int run_rank(const rtxh::CliOptions& o, void* hs, int rank, int nranks, Rendezvous* rv) {
  const int tile = o.tile > 0 ? o.tile : 16;
  if (rank == 0) {
    ncclUniqueId id;
    const ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) {
      rv->id_ready.store(-1);
      std::cerr << "rank 0: ncclGetUniqueId: " << ncclGetErrorString(r) << std::endl;
      return 3;
    }
    rv->uid = id;
    rv->id_ready.store(1, std::memory_order_release);
  } else {
    const auto t0 = std::chrono::steady_clock::now();
    while (rv->id_ready.load(std::memory_order_acquire) == 0) {
      if (waited_too_long(t0)) {
        std::cerr << "rank " << rank << ": no communicator id from rank 0" << std::endl;
        return 3;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    if (rv->id_ready.load() < 0) return 3;
  }
  // everything up to the communicator: a failure is published (rendezvous)
  auto early = [&](int code) {
    rv->failed.store(1);
    return code;
  };
  const int device = o.device + rank;
  int ndev = 0;
  if (rtx_device_count(&ndev) != RTX_OK || device >= ndev) {
    std::cerr << "rank " << rank << ": no GPU " << device << " (" << ndev << " visible)" << std::endl;
    return early(2);
  }
  RtxSceneDesc desc;
  rtx_host_desc(hs, &desc);
  RtxHostInfo info;
  rtx_host_info(hs, &info);
  void* scene = nullptr;
  if (rtx_scene_create(device, &desc, &scene) != RTX_OK) {
    std::cerr << "rank " << rank << ": rtx: " << rtx_last_error() << std::endl;
    return early(2);
  }
  if (hipSetDevice(device) != hipSuccess) {
    std::cerr << "rank " << rank << ": hipSetDevice failed" << std::endl;
    return early(3);
  }
  hipStream_t stream;
  if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) {
    std::cerr << "rank " << rank << ": hipStreamCreate failed" << std::endl;
    return early(3);
  }

  const int width = o.size;
  const int height = rtx_image_height(width, info.aspect);
  RtxRenderParams p = rtxh::cli_params(o, width, height);
  p.tile = tile;
  p.shard = rank;
  p.nshards = nranks;
  p.packed = 1;
  // ncclGather moves equal counts: every shard padded to the largest
  std::vector<int64_t> npix(nranks);
  int64_t maxpix = 0;
  for (int r = 0; r < nranks; ++r) {
    RtxRenderParams q = p;
    q.shard = r;
    rtx_shard_pixels(&q, &npix[r]);
    maxpix = std::max(maxpix, npix[r]);
  }
  const size_t shard_bytes = size_t(maxpix) * 3;
  uint8_t* d_send = nullptr;
  uint8_t* d_recv = nullptr;
  if (hipMalloc(&d_send, shard_bytes > 0 ? shard_bytes : 1) != hipSuccess ||
      hipMemsetAsync(d_send, 0, shard_bytes, stream) != hipSuccess ||
      (rank == 0 && hipMalloc(&d_recv, shard_bytes * nranks > 0 ? shard_bytes * nranks : 1) != hipSuccess)) {
    std::cerr << "rank " << rank << ": device buffers: out of memory" << std::endl;
    return early(3);
  }
  if (!rendezvous_join(rv, rank, nranks)) return 3;
  ncclComm_t comm;
  NCCL_CHECK(ncclCommInitRank(&comm, nranks, rv->uid, rank), "ncclCommInitRank");
  RtxStats st;
  HIP_CHECK(hipStreamSynchronize(stream), "hipStreamSynchronize");
  const auto t0 = std::chrono::steady_clock::now();
  if (rtx_render(scene, &p, d_send, nullptr, nullptr, 1, stream, o.stats ? &st : nullptr) != RTX_OK) {
    std::cerr << "rank " << rank << ": rtx: " << rtx_last_error() << std::endl;
    return 2;
  }
  NCCL_CHECK(ncclGather(d_send, d_recv, shard_bytes, ncclUint8, 0, comm, stream), "ncclGather");
  HIP_CHECK(hipStreamSynchronize(stream), "hipStreamSynchronize");
  // the device-buffer render's outcome (rtx_frame_status): a frame known to
  // be wrong fails the rank, and with it the job
  if (rtx_frame_status(scene, nullptr, nullptr) != RTX_OK) {
    std::cerr << "rank " << rank << ": rtx: " << rtx_last_error() << std::endl;
    return 2;
  }
  rv->rank_ms[rank % 64] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  rv->rank_rays[rank % 64] = o.stats ? st.rays : 0;
  int rc = 0;
  if (rank == 0) {
    std::vector<uint8_t> packed(shard_bytes * nranks);
    HIP_CHECK(hipMemcpy(packed.data(), d_recv, packed.size(), hipMemcpyDeviceToHost), "hipMemcpy");
    std::vector<uint8_t> frame(size_t(width) * height * 3, 0);
    for (int r = 0; r < nranks; ++r)
      if (rtx_unpack_tiles(packed.data() + shard_bytes * r, width, height, tile, r, nranks, 3, frame.data()) != RTX_OK)
        rc = 1;
    if (rtx_write_image(o.img_name.c_str(), width, height, frame.data()) != RTX_OK) {
      std::cerr << rtx_host_last_error() << std::endl;
      rc = 1;
    }
  }
  ncclCommDestroy(comm);
  (void)hipFree(d_send);
  if (d_recv) (void)hipFree(d_recv);
  (void)hipStreamDestroy(stream);
  rtx_scene_destroy(scene);
  return rc;
}

}  // namespace

// Runs the sharded render; returns the process exit code (0, or the first
// failing rank's).  hs: the parsed scene (rtx_host_load).
int rtx_cli_multi_gpu(const rtxh::CliOptions& o, void* hs) {
  const int n = o.gpus;
  if (n < 1 || n > 64) {
    std::cerr << "--gpus must be in [1, 64]" << std::endl;
    return 1;
  }
  void* page = mmap(nullptr, sizeof(Rendezvous), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  if (page == MAP_FAILED) {
    std::perror("mmap");
    return 1;
  }
  Rendezvous* rv = new (page) Rendezvous();
  rv->id_ready.store(0);
  rv->joined.store(0);
  rv->failed.store(0);
  std::vector<pid_t> kids;
  const auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < n; ++r) {
    std::cout.flush();
    std::cerr.flush();
    const pid_t pid = fork();
    if (pid < 0) {
      std::perror("fork");
      for (pid_t k : kids) kill(k, SIGTERM);
      return 1;
    }
    if (pid == 0) {
      const int rc = run_rank(o, hs, r, n, rv);
      std::cout.flush();
      std::cerr.flush();
      _exit(rc);
    }
    kids.push_back(pid);
  }
  // Reap the ranks in the order they end.  The first rank to fail ends the
  // job: the others may be blocked in a collective waiting for it, so they
  // get SIGTERM, then SIGKILL after a grace period; the job returns the
  // failing rank's status.
  int rc = 0;
  std::vector<bool> alive(kids.size(), true);
  size_t left = kids.size();
  bool terminating = false;
  auto kill_rest = [&](int sig) {
    for (size_t r = 0; r < kids.size(); ++r)
      if (alive[r]) kill(kids[r], sig);
  };
  auto t_term = std::chrono::steady_clock::now();
  while (left > 0) {
    int status = 0;
    const pid_t pid = waitpid(-1, &status, terminating ? WNOHANG : 0);
    if (pid < 0) {
      if (errno == EINTR) continue;
      rc = rc ? rc : 1;
      break;
    }
    if (pid == 0) {  // terminating: ranks still running
      if (std::chrono::steady_clock::now() - t_term > std::chrono::seconds(10)) {
        kill_rest(SIGKILL);
        terminating = false;  // block until they are reaped
      } else {
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
      }
      continue;
    }
    size_t r = 0;
    while (r < kids.size() && kids[r] != pid) ++r;
    if (r == kids.size()) continue;
    alive[r] = false;
    --left;
    const int code = WIFEXITED(status) ? WEXITSTATUS(status) : 128 + (WIFSIGNALED(status) ? WTERMSIG(status) : 0);
    if (code != 0 && rc == 0) {
      rc = code;
      if (left > 0) {
        std::cerr << "rank " << r << " failed (status " << code << "): ending the other ranks" << std::endl;
        rv->failed.store(1);
        kill_rest(SIGTERM);
        terminating = true;
        t_term = std::chrono::steady_clock::now();
      }
    }
  }
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (o.stats && rc == 0) {
    double worst = 0.0;
    long long rays = 0;
    for (int r = 0; r < n && r < 64; ++r) {
      worst = std::max(worst, rv->rank_ms[r]);
      rays += rv->rank_rays[r];
    }
    std::printf("{\"backend\": \"hip-gfx950\", \"gpus\": %d, \"ms\": %.3f, \"render_gather_ms\": %.3f, \"rays\": %lld, "
                "\"mrays_per_s\": %.3f}\n",
                n, ms, worst, rays, worst > 0 ? rays / worst / 1e3 : 0.0);
  }
  munmap(page, sizeof(Rendezvous));
  return rc;
}

#include "xgmi_comm.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>

#include <rccl/rccl.h>

#include "kernels/common.h"

namespace {
std::string handle_bytes(const hipIpcMemHandle_t& h) {
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}
hipIpcMemHandle_t handle_from(const std::string& b) {
  if (b.size() != sizeof(hipIpcMemHandle_t))
    throw std::runtime_error("XgmiComm: IPC handle of " + std::to_string(b.size()) + " bytes");
  hipIpcMemHandle_t h;
  std::memcpy(&h, b.data(), sizeof(h));
  return h;
}
}  // namespace

XgmiComm::XgmiComm(int nranks, int rank, bool emulate, double lat_us, double link_gbps,
                   double timeout_s)
    : nranks_(nranks), rank_(rank), emulate_(emulate) {
  if (nranks < 1 || nranks > xgmi::kMaxRanks || rank < 0 || rank >= nranks)
    throw std::runtime_error("XgmiComm: 1..8 ranks on one xGMI node");
  if (emulate && rank != 0) throw std::runtime_error("XgmiComm: an emulated comm is rank 0");
  // uncached: remote flag stores must be seen by the local polls (no L2 copy)
  HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&flags_),
                                  xgmi::kFlagWords * sizeof(unsigned), hipDeviceMallocUncached));
  HIP_CHECK(hipMemset(flags_, 0, xgmi::kFlagWords * sizeof(unsigned)));
  HIP_CHECK(hipMalloc(&epoch_, xgmi::kMaxBlocks * sizeof(unsigned)));
  HIP_CHECK(hipMemset(epoch_, 0, xgmi::kMaxBlocks * sizeof(unsigned)));
  HIP_CHECK(hipMalloc(&error_, sizeof(unsigned)));
  HIP_CHECK(hipMemset(error_, 0, sizeof(unsigned)));
  HIP_CHECK(hipDeviceSynchronize());
  sync_.nranks = nranks;
  sync_.rank = rank;
  sync_.flags = flags_;
  sync_.peer_flags[rank] = flags_;
  sync_.epoch = epoch_;
  sync_.error = error_;
  sync_.emulate = emulate ? 1 : 0;
  sync_.timeout_ticks = (long long)(timeout_s * 1e8);
  if (emulate) {
    sync_.lat_ticks = (long long)(lat_us * 100.0);
    // 1 MiB at link_gbps GB/s, in 100 MHz ticks
    sync_.link_ticks_per_mib =
        link_gbps > 0 ? (long long)(1048576.0 / (link_gbps * 1e9) * 1e8 + 0.5) : 0;
    for (int r = 0; r < nranks; ++r) sync_.peer_flags[r] = flags_;
  }
}

XgmiComm::~XgmiComm() {
  for (auto& kv : opened_) (void)hipIpcCloseMemHandle(kv.second);
  for (void* p : opened_flags_) (void)hipIpcCloseMemHandle(p);
  for (void* p : emu_allocs_) (void)hipFree(p);
  if (flags_) (void)hipFree(flags_);
  if (epoch_) (void)hipFree(epoch_);
  if (error_) (void)hipFree(error_);
}

std::string XgmiComm::flags_handle() const {
  hipIpcMemHandle_t h;
  HIP_CHECK(hipIpcGetMemHandle(&h, flags_));
  return handle_bytes(h);
}

void XgmiComm::open_flags(int r, const std::string& handle) {
  if (r < 0 || r >= nranks_) throw std::runtime_error("XgmiComm: bad peer rank");
  if (r == rank_ || emulate_) return;
  void* p = nullptr;
  const hipIpcMemHandle_t h = handle_from(handle);
  HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  opened_flags_.push_back(p);
  sync_.peer_flags[r] = static_cast<unsigned*>(p);
}

std::pair<std::string, size_t> XgmiComm::export_buffer(uintptr_t ptr, size_t bytes) const {
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  HIP_CHECK(hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(ptr)));
  const size_t off = ptr - reinterpret_cast<uintptr_t>(base);
  if (off + bytes > size) throw std::runtime_error("XgmiComm: buffer crosses its allocation");
  hipIpcMemHandle_t h;
  HIP_CHECK(hipIpcGetMemHandle(&h, base));
  return {handle_bytes(h), off};
}

void* XgmiComm::open_handle(int r, const std::string& handle) {
  auto key = std::make_pair(r, handle);
  auto it = opened_.find(key);
  if (it != opened_.end()) return it->second;
  void* p = nullptr;
  HIP_CHECK(hipIpcOpenMemHandle(&p, handle_from(handle), hipIpcMemLazyEnablePeerAccess));
  opened_[key] = p;
  return p;
}

XgmiComm::Reg& XgmiComm::reg_for(uintptr_t local, size_t bytes) {
  for (Reg& g : regs_)
    if (g.local == local) {
      if (g.bytes != bytes) throw std::runtime_error("XgmiComm: buffer re-registered with another size");
      return g;
    }
  Reg g;
  g.local = local;
  g.bytes = bytes;
  g.peer[rank_] = reinterpret_cast<void*>(local);
  regs_.push_back(g);
  return regs_.back();
}

void XgmiComm::open_buffer(uintptr_t local, size_t bytes, int r, const std::string& handle,
                           size_t off) {
  if (r < 0 || r >= nranks_) throw std::runtime_error("XgmiComm: bad peer rank");
  Reg& g = reg_for(local, bytes);
  if (r == rank_) return;
  g.peer[r] = static_cast<char*>(open_handle(r, handle)) + off;
}

void XgmiComm::emulate_buffer(uintptr_t local, size_t bytes) {
  if (!emulate_) throw std::runtime_error("XgmiComm: emulate_buffer on a real communicator");
  Reg& g = reg_for(local, bytes);
  for (int r = 0; r < nranks_; ++r) {
    if (r == rank_ || g.peer[r]) continue;
    void* p = nullptr;
    HIP_CHECK(hipMalloc(&p, bytes));
    HIP_CHECK(hipMemcpy(p, reinterpret_cast<void*>(local), bytes, hipMemcpyDeviceToDevice));
    emu_allocs_.push_back(p);
    g.peer[r] = p;
  }
}

bool XgmiComm::ready() const {
  for (int r = 0; r < nranks_; ++r)
    if (!sync_.peer_flags[r]) return false;
  return true;
}

const XgmiComm::Reg* XgmiComm::find(const void* p, size_t bytes) const {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  for (const Reg& g : regs_)
    if (a >= g.local && a + bytes <= g.local + g.bytes) {
      for (int r = 0; r < nranks_; ++r)
        if (!g.peer[r]) return nullptr;
      return &g;
    }
  return nullptr;
}

bool XgmiComm::registered(const void* local, size_t bytes) const {
  return find(local, bytes) != nullptr;
}

void* XgmiComm::peer_ptr(const void* local, int r) const {
  const Reg* g = find(local, 1);
  if (!g || r < 0 || r >= nranks_)
    throw std::runtime_error("XgmiComm: address outside every registered buffer");
  return static_cast<char*>(g->peer[r]) + (reinterpret_cast<uintptr_t>(local) - g->local);
}

unsigned XgmiComm::error() const {
  unsigned v = 0;
  HIP_CHECK(hipDeviceSynchronize());
  HIP_CHECK(hipMemcpy(&v, error_, sizeof(v), hipMemcpyDeviceToHost));
  return v;
}

void XgmiComm::clear_error() {
  HIP_CHECK(hipDeviceSynchronize());
  HIP_CHECK(hipMemset(error_, 0, sizeof(unsigned)));
}

void XgmiComm::all_reduce(const void* send, void* recv, size_t count, int dtype, int op,
                          hipStream_t s) {
  if (send != recv || dtype != ncclFloat32 || op != ncclSum)
    throw std::runtime_error("XgmiComm::all_reduce: in-place fp32 sum only");
  launch(recv, count, false, s);
}

void XgmiComm::gather_segments(void* buf, size_t count, hipStream_t s) {
  launch(buf, count, true, s);
}

void XgmiComm::all_reduce_sgd(float* grads, float* params, float* mom, size_t count,
                              long long l2_end, float l2, float momentum, float gscale,
                              const float* lr, long long* step, hipStream_t s) {
  if (!mom || !lr || l2_end % 4) throw std::runtime_error("XgmiComm::all_reduce_sgd: arguments");
  if (!registered(params, count * sizeof(float)))
    throw std::runtime_error("XgmiComm::all_reduce_sgd: params not registered");
  xgmi::AllReduceArgs a;
  for (int r = 0; r < nranks_; ++r) a.w[r] = static_cast<float*>(peer_ptr(params, r));
  a.mom = mom;
  a.lr = lr;
  a.momentum = momentum;
  a.gscale = gscale;
  a.l2 = l2;
  a.l2_end4 = l2_end / 4;
  a.step = step;
  launch(grads, count, false, s, &a);
}

void XgmiComm::all_reduce_sgd_oneshot(const float* grads2, float* params, float* mom,
                                      size_t count, float momentum, float gscale, const float* lr,
                                      long long* step, unsigned* done, hipStream_t s) {
  if (count == 0 || count % 4) throw std::runtime_error("XgmiComm::all_reduce_sgd_oneshot: count");
  if (!ready()) throw std::runtime_error("XgmiComm: flags of some rank not mapped");
  if (!registered(grads2, 2 * count * sizeof(float)))
    throw std::runtime_error("XgmiComm::all_reduce_sgd_oneshot: grads2 [2][count] not registered");
  xgmi::OneShotArgs a;
  a.s = sync_;
  for (int r = 0; r < nranks_; ++r) a.g[r] = static_cast<const float*>(peer_ptr(grads2, r));
  a.w = params;
  a.mom = mom;
  a.n4 = (long long)(count / 4);
  a.lr = lr;
  a.momentum = momentum;
  a.gscale = gscale;
  a.step = step;
  a.done = done;
  xgmi::launch_oneshot_sgd(a, s);
}

void XgmiComm::emulate_fill_peer(uintptr_t local, int r, uintptr_t src, size_t bytes) {
  if (!emulate_) throw std::runtime_error("XgmiComm: emulate_fill_peer on a real communicator");
  const Reg* g = find(reinterpret_cast<const void*>(local), bytes);
  if (!g || r < 0 || r >= nranks_) throw std::runtime_error("XgmiComm: emulate_fill_peer target");
  HIP_CHECK(hipMemcpy(peer_ptr(reinterpret_cast<const void*>(local), r),
                      reinterpret_cast<const void*>(src), bytes, hipMemcpyDeviceToDevice));
}

void XgmiComm::launch(void* recv, size_t count, bool gather_only, hipStream_t s,
                      const xgmi::AllReduceArgs* sgd, float* out) {
  if (count == 0) return;
  if (count % 4) throw std::runtime_error("XgmiComm::all_reduce: count must be a multiple of 4");
  if (!ready()) throw std::runtime_error("XgmiComm: flags of some rank not mapped");
  const size_t bytes = count * sizeof(float);
  if (!registered(recv, bytes)) throw std::runtime_error("XgmiComm::all_reduce: unregistered buffer");
  xgmi::AllReduceArgs a;
  if (sgd) a = *sgd;
  a.s = sync_;
  for (int r = 0; r < nranks_; ++r) a.buf[r] = static_cast<float*>(peer_ptr(recv, r));
  a.n4 = (long long)(count / 4);
  a.seg4 = (a.n4 + nranks_ - 1) / nranks_;
  a.out = out;
  // Grid: <= 256 blocks (64 when the ranks share a GPU: a block waiting at a
  // barrier holds its CU slot).  Segments under 256 float4s a block at that
  // grid (LeNet-5's 62 K floats: 1,938 float4s a segment at N = 8) take
  // 64-thread blocks of >= 64 float4s, so the grid stays wide instead of
  // collapsing to a few 256-thread blocks that walk the segment serially; a
  // thread keeps kAllReduceUnroll float4s of every rank in flight.
  const long long nb = sync_.lean ? 64 : 256;
  const long long per = (a.seg4 + nb - 1) / nb;
  const int nt = per >= 512 ? 256 : 64;
  const long long gran = nt * 2LL;  // one unrolled pass of the block
  const long long per4 = std::max<long long>(nt, (per + gran - 1) / gran * gran);
  a.per4 = (int)per4;
  a.link_bytes = a.seg4 * 16;
  a.gather_only = gather_only ? 1 : 0;
  const int blocks = (int)std::max<long long>(1, (a.seg4 + per4 - 1) / per4);
  xgmi::launch_allreduce(a, blocks, nt, s);
}

void XgmiComm::all_gather(const void* send, void* recv, size_t send_count, int dtype,
                          hipStream_t s) {
  if (dtype != ncclFloat32 || send_count % 4)
    throw std::runtime_error("XgmiComm::all_gather: fp32, a multiple of 4 floats a rank");
  float* mine = static_cast<float*>(recv) + (size_t)rank_ * send_count;
  if (send != mine)  // the peers read this rank's slot of ITS recv buffer
    HIP_CHECK(hipMemcpyAsync(mine, send, send_count * sizeof(float), hipMemcpyDeviceToDevice, s));
  launch(recv, send_count * nranks_, true, s);
}

void XgmiComm::reduce_scatter(const void* send, void* recv, size_t recv_count, int dtype, int op,
                              hipStream_t s) {
  if (dtype != ncclFloat32 || op != ncclSum || recv_count % 4)
    throw std::runtime_error("XgmiComm::reduce_scatter: fp32 sum, a multiple of 4 floats a rank");
  // the send buffer is what the peers read (registered).  The reduced
  // segment is a plain local store into recv: in place (recv = this rank's
  // slot of send) is safe, since the peers read only the OTHER slots of it
  launch(const_cast<void*>(send), recv_count * nranks_, false, s, nullptr,
         static_cast<float*>(recv));
}

#include "collective.h"

#include <stdexcept>

size_t dtype_bytes(int dtype) {
  switch (dtype) {  // ncclDataType_t values (rccl.h)
    case 0:         // int8
    case 1:         // uint8
      return 1;
    case 6:  // float16
    case 9:  // bfloat16
      return 2;
    case 2:  // int32
    case 3:  // uint32
    case 7:  // float32
      return 4;
    case 4:  // int64
    case 5:  // uint64
    case 8:  // float64
      return 8;
    default:
      throw std::runtime_error("EmuComm: unsupported dtype");
  }
}

EmuComm::EmuComm(int nranks, int rank, double lat_us, double busbw_gbps, int blocks)
    : nranks_(nranks), rank_(rank), blocks_(blocks), lat_us_(lat_us), busbw_(busbw_gbps) {
  if (nranks < 1 || rank < 0 || rank >= nranks || busbw_gbps <= 0 || blocks < 1)
    throw std::runtime_error("EmuComm: bad configuration");
}

double EmuComm::all_reduce_us(size_t bytes) const {
  const double n = nranks_;
  return lat_us_ + 2.0 * (n - 1) / n * (double)bytes / (busbw_ * 1e3);
}

double EmuComm::gather_us(size_t full_bytes) const {
  const double n = nranks_;
  return lat_us_ + (n - 1) / n * (double)full_bytes / (busbw_ * 1e3);
}

double EmuComm::lat_once() {
  if (!in_group_) return lat_us_;
  return grouped_++ == 0 ? lat_us_ : 0.0;
}

void EmuComm::occupy(void* buf, size_t bytes, double us, hipStream_t s) {
  commemu::launch_occupy(buf, bytes, us, blocks_, s);
}

void EmuComm::all_reduce(const void*, void* recv, size_t count, int dtype, int, hipStream_t s) {
  const size_t b = count * dtype_bytes(dtype);
  occupy(recv, b, all_reduce_us(b) - lat_us_ + lat_once(), s);
}

void EmuComm::all_gather(const void*, void* recv, size_t send_count, int dtype, hipStream_t s) {
  const size_t b = send_count * dtype_bytes(dtype) * (size_t)nranks_;
  occupy(recv, b, gather_us(b) - lat_us_ + lat_once(), s);
}

void EmuComm::reduce_scatter(const void* send, void*, size_t recv_count, int dtype, int,
                             hipStream_t s) {
  const size_t b = recv_count * dtype_bytes(dtype) * (size_t)nranks_;
  occupy(const_cast<void*>(send), b, gather_us(b) - lat_us_ + lat_once(), s);
}

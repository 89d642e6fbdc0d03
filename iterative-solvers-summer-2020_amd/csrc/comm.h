// Row-slab communicators: RCCL over xGMI (one process per GPU) and a loopback group (several
// slabs on one GPU, one host thread each) that exercises the same slab logic on a single device.
//
// The reference has no distributed code at all; the exchange pattern is
// the one the periodic 13-point stencil needs: a 2-row halo with the up/down ring neighbours per
// stencil pass, plus small all-reduces (sum for dots / norms, max for the max-norm of
// TerminationCondition, scipy/optimize/_nonlin.py:354).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/nkhip.h"

namespace nk {
struct PeerArgs;  // peer_dev.h
}

// Halo slots of the pushed-halo-rows path (peer-memory communicator): this rank's slot region
// and its ring neighbours' (mapped peer memory); slot q = 4 rows of `ld` doubles at base + 4 q ld
// (rows 0, 1: the previous rank's last two rows of pool vector q, rows 2, 3: the next rank's
// first two).
struct nk_halo_slots {
  double* mine = nullptr;
  double* prev = nullptr;
  double* next = nullptr;
  int64_t ld = 0, count = 0;
};

struct nk_comm {
  virtual ~nk_comm() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  // dev[0, nsum) summed and dev[nsum, nv) max-reduced over ranks, in place in device memory,
  // ordered on `s` (RCCL: enqueued, no host synchronisation).  Returns 0 or a negative NK_E* code.
  virtual int allreduce(double* dev, int nsum, int nv, hipStream_t s) = 0;
  // The same, with the result also in `host` (pinned host memory) once the stream reaches it:
  // here a D2H copy ordered after the all-reduce; the peer-memory communicator's kernel writes
  // it itself (allreduce_writes_host: no runtime blit, and the host may poll the slot).
  virtual int allreduce_host(double* dev, double* host, int nsum, int nv, hipStream_t s) {
    const int rc = allreduce(dev, nsum, nv, s);
    if (rc) return rc;
    return hipMemcpyAsync(host, dev, sizeof(double) * nv, hipMemcpyDeviceToHost, s) == hipSuccess
               ? NK_OK
               : NK_EHIP;
  }
  virtual bool allreduce_writes_host() const { return false; }
  // lo <- rows ny_prev-2, ny_prev-1 of the previous rank, hi <- rows 0, 1 of the next rank
  // (periodic ring).  Enqueued on `s` (RCCL) or completed before return (loopback).
  virtual int halo(const double* v, double* lo, double* hi, int64_t ny, int64_t nx,
                   hipStream_t s) = 0;
  virtual int barrier(hipStream_t s) = 0;
  // A rank that fails outside the collective calls (a HIP error, an exception in its host
  // thread) marks the group aborted: peers blocked in (or entering) a collective return
  // NK_ECOMM instead of waiting forever.  RCCL: ncclCommAbort.
  virtual void abort() = 0;
  // the ranks' kernels share one device (loopback): launches of different ranks run
  // concurrently, so a kernel cannot count on its whole grid being resident
  virtual bool shares_device() const { return false; }
  // some two ranks of the group share a device (the same answer on every rank)
  virtual bool group_shares_device() const { return shares_device(); }
  // a collective already enqueued on the device failed (peer-memory communicator: a wait timed
  // out or the group was aborted); checked after each stream synchronisation (Engine::sync)
  virtual bool failed() const { return false; }
  // Peer-memory communicator only: the arguments of the NEXT all-reduce of nv values / halo
  // exchange of nx columns, for a kernel that runs the collective inside its own launch
  // (arnctl.hip: reduction + all-reduce + Arnoldi control; arnoldi.hip: slab edge rows + halo).
  // The collective's tag advances exactly as allreduce() / halo() would advance it, so every
  // rank must take the same sequence.  false: not available (the caller uses allreduce / halo).
  virtual bool take_allreduce(nk::PeerArgs* /*out*/, int /*nv*/) { return false; }
  virtual bool take_halo(nk::PeerArgs* /*out*/, int64_t /*nx*/) { return false; }
  // The halo slots, for one stepper at a time (`owner`); false: none (not the peer-memory
  // communicator, or another stepper holds them).  release_slots hands them back.
  virtual bool claim_slots(const void* /*owner*/, nk_halo_slots* /*out*/) { return false; }
  // All-reduces this rank has issued so far (every rank counts the same sequence): a write into
  // the neighbours' halo slots issued before all-reduce e is visible to every rank's launches
  // issued after it, i.e. once epoch() > e.
  virtual uint64_t epoch() const { return 0; }
  virtual void release_slots(const void* /*owner*/) {}
};

namespace nk {
int comm_unique_id_bytes();
int comm_get_unique_id(void* out);
int comm_create_rccl(nk_comm** out, const void* uid, int rank, int nranks);
int comm_create_loopback(nk_comm** out, int nranks);
// peer-memory communicator (peer.hip): create (allocate + export this rank's buffer, write its
// handle blob), then connect with every rank's blob (rank order)
int comm_peer_handle_bytes();
int comm_create_peer(nk_comm** out, int rank, int nranks, int64_t max_nx, void* handle_out);
int comm_peer_connect(nk_comm* c, const void* handles);
}  // namespace nk

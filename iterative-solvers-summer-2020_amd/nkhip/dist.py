"""Row-slab decomposition of the periodic grid over GPUs (RCCL over xGMI).

The reference is single-process (no MPI/NCCL/Gloo anywhere).  Here the
N x N torus is cut into row slabs, one per rank (one process per GPU):

* rank p owns rows [row0(p), row0(p) + ny(p)); x stays periodic inside the slab;
* every stencil pass reads a 2-row halo from the up/down ring neighbours (grouped
  ncclSend/ncclRecv issued by libnkhip on the solver's stream);
* dots, norms and max-norms of the Newton-Krylov loop are all-reduced (sum / max) once per
  fused reduction, so every rank runs the identical host-side Hessenberg algebra.

``slab_rows`` is plain arithmetic (tested on CPU); ``RcclComm.from_torch_distributed`` shares
the RCCL unique id through an initialised ``torch.distributed`` process group (gloo or nccl);
``PeerComm.from_torch_distributed`` exchanges the peer-memory buffers' IPC handles the same way.
"""
from __future__ import annotations

import ctypes as C

from ._lib import check, lib


def slab_rows(ny_global: int, rank: int, nranks: int):
    """(row0, ny_local) of rank's slab: balanced, every slab >= 2 rows (the halo depth)."""
    if nranks < 1 or not 0 <= rank < nranks:
        raise ValueError("bad rank / nranks")
    base, extra = divmod(int(ny_global), int(nranks))
    ny = base + (1 if rank < extra else 0)
    row0 = rank * base + min(rank, extra)
    if nranks > 1 and ny < 2:
        raise ValueError(f"{ny_global} rows cannot give {nranks} slabs of >= 2 rows")
    return row0, ny


def neighbours(rank: int, nranks: int):
    """(prev, next) ranks on the periodic ring: prev owns the rows above, next the rows below."""
    return (rank - 1) % nranks, (rank + 1) % nranks


class Comm:
    def __init__(self, handle, rank, size):
        self.handle = handle
        self.rank = rank
        self.size = size

    def abort(self):
        """Mark the group failed: peers blocked in a collective return NK_ECOMM (nk_comm_abort).
        A host thread driving a slab calls this when it fails, before it exits."""
        if self.handle:
            lib.nk_comm_abort(self.handle)

    def close(self):
        if self.handle:
            lib.nk_comm_destroy(self.handle)
            self.handle = None

    def selftest(self, nx: int = 64) -> bool:
        """A collective (every rank calls it): one all-reduce and one halo exchange of known
        values through the group, checked on the host (nk_comm_selftest).  False: a value did
        not arrive intact or a wait gave up."""
        import torch
        stream = torch.cuda.current_stream().cuda_stream
        return lib.nk_comm_selftest(self.handle, int(nx), C.c_void_p(stream)) == 0

    def selftest_push(self, nx: int = 64):
        """A collective: the pushed-halo-rows protocol of the slab solver (push into the
        neighbours' halo slots, one all-reduce, read back, host check; nk_comm_selftest_push).
        True / False (a row did not arrive intact or a wait gave up), or None when the group has
        no halo slots to check (RCCL, or a stepper holds them) -- the same answer on every rank
        except for False, which the caller must agree on over its side channel."""
        import torch
        stream = torch.cuda.current_stream().cuda_stream
        rc = lib.nk_comm_selftest_push(self.handle, int(nx), C.c_void_p(stream))
        return None if rc == -1 else rc == 0


class RcclComm(Comm):
    @staticmethod
    def unique_id() -> bytes:
        n = lib.nk_comm_unique_id_bytes()
        buf = (C.c_char * n)()
        check(lib.nk_comm_get_unique_id(buf), "nk_comm_get_unique_id")
        return bytes(buf)

    @classmethod
    def create(cls, uid: bytes, rank: int, nranks: int) -> "RcclComm":
        h = C.c_void_p()
        buf = (C.c_char * len(uid)).from_buffer_copy(uid)
        check(lib.nk_comm_create_rccl(C.byref(h), buf, int(rank), int(nranks)),
              "nk_comm_create_rccl")
        return cls(h, rank, nranks)

    @classmethod
    def from_torch_distributed(cls) -> "RcclComm":
        import torch.distributed as dist
        rank, size = dist.get_rank(), dist.get_world_size()
        obj = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        return cls.create(obj[0], rank, size)


class PeerComm(Comm):
    """Peer-memory communicator (csrc/peer.hip): every rank exports one fine-grained device
    buffer; halos and all-reduces are single small kernels that write into the peers' buffers
    over xGMI and wait for tagged flags -- no RCCL call on the solver's stream.  One PROCESS per
    rank: one process per GPU, or several processes on one GPU (IPC on the same device).  Ranks
    as threads of one process are refused (nk_comm_peer_connect returns NK_EINVAL): they share
    the process's in-order hardware queues, so a collective waiting for a peer rank could sit
    ahead of the very launch it waits for.  ``max_nx``: the widest slab row any collective will
    carry."""

    def __init__(self, handle, rank, size, blob=b""):
        super().__init__(handle, rank, size)
        self.blob = blob

    @classmethod
    def create(cls, rank: int, nranks: int, max_nx: int) -> "PeerComm":
        h = C.c_void_p()
        buf = (C.c_char * lib.nk_comm_peer_handle_bytes())()
        check(lib.nk_comm_create_peer(C.byref(h), int(rank), int(nranks), int(max_nx), buf),
              "nk_comm_create_peer")
        return cls(h, rank, nranks, bytes(buf))

    def connect(self, blobs):
        """Map every rank's buffer (``blobs``: each rank's ``blob``, in rank order)."""
        allb = b"".join(blobs)
        buf = (C.c_char * len(allb)).from_buffer_copy(allb)
        check(lib.nk_comm_peer_connect(self.handle, buf), "nk_comm_peer_connect")
        return self

    @classmethod
    def from_torch_distributed(cls, max_nx: int, group=None) -> "PeerComm":
        """Create this rank's side and exchange the handle blobs through an initialised
        torch.distributed group (any backend)."""
        import torch.distributed as dist
        rank, size = dist.get_rank(group), dist.get_world_size(group)
        c = cls.create(rank, size, max_nx)
        blobs = [None] * size
        dist.all_gather_object(blobs, c.blob, group=group)
        return c.connect(blobs)


def peer_comms(nranks: int, max_nx: int):
    """A peer-memory group inside this process: only a world of one (the rank is its own ring
    neighbour; tests, bench.py --peer-self).  Several ranks need one process each
    (PeerComm.from_torch_distributed)."""
    if nranks != 1:
        raise ValueError("a peer-memory group takes one process per rank: build it with "
                         "PeerComm.from_torch_distributed in each rank's process")
    cs = [PeerComm.create(r, nranks, max_nx) for r in range(nranks)]
    blobs = [c.blob for c in cs]
    for c in cs:
        c.connect(blobs)
    return cs


def loopback_comms(nranks: int):
    """``nranks`` slabs on the current GPU, each to be stepped from its own host thread."""
    arr = (C.c_void_p * nranks)()
    check(lib.nk_comm_create_loopback(arr, int(nranks)), "nk_comm_create_loopback")
    return [Comm(C.c_void_p(arr[i]), i, nranks) for i in range(nranks)]

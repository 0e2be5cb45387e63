"""A torch-free host exchange for the ranks of one job (TCP star through rank 0).

It carries what the ranks need before (and beside) RCCL: the 128-byte RCCL unique id from rank 0
to every rank, and — when ranks share a device, where RCCL takes one rank per GPU — libycrdt's own
collectives as host callbacks (ycrdt_comm_create_exchange: all-reduce of u32 words, all-gather of
equal-length byte strings). crdt.js's ranks are Node processes; this is the same shape as the
router's own peer sockets, and nothing here imports torch.

    hub = HostHub(world, rank, "127.0.0.1", port)   # rank 0 listens on port, the others connect
    uid = hub.bcast(Comm.unique_id() if rank == 0 else None)
    comm = Comm(engine, world, rank, uid)            # RCCL, one rank per GPU
    comm = Comm.over_hub(engine, hub)                # or the library's collectives over the hub

Trust model: the hub is a job-internal channel. Bind it to loopback or a trusted interface. Every
rank sends a job token in its handshake (YCRDT_HUB_TOKEN, else a token derived from the launcher's
MASTER_ADDR / MASTER_PORT), and rank 0 drops a connection whose token or rank is wrong. Frames are
capped at YCRDT_HUB_MAX_FRAME bytes (default 4 GiB), so a peer cannot make a rank allocate more.
"""
import hashlib
import os
import socket
import struct
import time

import numpy as np

_HDR = struct.Struct("<Q")
_MAX_FRAME = int(os.environ.get("YCRDT_HUB_MAX_FRAME", str(4 << 30)))


def _job_token(addr: str, port: int) -> bytes:
    tok = os.environ.get("YCRDT_HUB_TOKEN")
    if tok is None:
        tok = f"ycrdt-hub:{os.environ.get('MASTER_ADDR', addr)}:{os.environ.get('MASTER_PORT', port)}"
    return hashlib.sha256(tok.encode()).digest()


def _send(sock, payload: bytes):
    sock.sendall(_HDR.pack(len(payload)) + payload)


def _recv_exact(sock, n: int) -> bytes:
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            raise ConnectionError("host hub: a rank closed its connection")
        got += k
    return bytes(buf)


def _recv(sock) -> bytes:
    (n,) = _HDR.unpack(_recv_exact(sock, _HDR.size))
    if n > _MAX_FRAME:
        raise ConnectionError(f"host hub: a {n}-byte frame exceeds the {_MAX_FRAME}-byte cap")
    return _recv_exact(sock, n)


class HostHub:
    """world ranks, rank 0 the hub. Every collective is entered by every rank in the same order."""

    def __init__(self, world: int, rank: int, addr: str, port: int, timeout: float = 300.0):
        self.world, self.rank = world, rank
        self._peers = {}
        self._sock = None
        if world == 1:
            return
        token = _job_token(addr, port)
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(world)
            srv.settimeout(timeout)
            try:
                while len(self._peers) < world - 1:
                    c, _ = srv.accept()
                    c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    c.settimeout(timeout)
                    try:
                        hello = _recv_exact(c, 4 + len(token))
                    except (OSError, ConnectionError):
                        c.close()
                        continue
                    (r,) = struct.unpack("<I", hello[:4])
                    if hello[4:] != token or not 0 < r < world or r in self._peers:
                        c.close()  # not a rank of this job: dropped, the hub keeps waiting
                        continue
                    self._peers[r] = c
            finally:
                srv.close()
        else:
            deadline = time.monotonic() + timeout
            while True:
                try:
                    s = socket.create_connection((addr, port), timeout=timeout)
                    break
                except OSError:
                    if time.monotonic() > deadline:
                        raise
                    time.sleep(0.05)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.sendall(struct.pack("<I", rank) + token)
            self._sock = s

    def allgather(self, payload: bytes) -> list:
        """Every rank's bytes (any lengths), in rank order."""
        payload = bytes(payload)
        if self.world == 1:
            return [payload]
        if self.rank == 0:
            parts = [payload] + [_recv(self._peers[r]) for r in range(1, self.world)]
            blob = b"".join(_HDR.pack(len(p)) + p for p in parts)
            for r in range(1, self.world):
                _send(self._peers[r], blob)
        else:
            _send(self._sock, payload)
            blob = _recv(self._sock)
        out, o = [], 0
        for _ in range(self.world):
            (n,) = _HDR.unpack_from(blob, o)
            o += _HDR.size
            out.append(blob[o:o + n])
            o += n
        return out

    def bcast(self, payload):
        """Rank 0's bytes on every rank."""
        return self.allgather(payload if self.rank == 0 else b"")[0]

    def allreduce_u32(self, a: np.ndarray, op: int):
        """In place over every rank: op 0 = sum (mod 2^32), 1 = max."""
        parts = self.allgather(a.astype(np.uint32).tobytes())
        arrs = [np.frombuffer(p, dtype=np.uint32) for p in parts]
        if op:
            a[:] = np.maximum.reduce(arrs)
        else:
            a[:] = (np.sum(np.stack(arrs).astype(np.uint64), axis=0) & 0xFFFFFFFF).astype(np.uint32)

    def barrier(self):
        self.allgather(b"")

    def close(self):
        for s in list(self._peers.values()) + ([self._sock] if self._sock else []):
            try:
                s.close()
            except OSError:
                pass
        self._peers, self._sock = {}, None

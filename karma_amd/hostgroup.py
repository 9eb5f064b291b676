"""Host-side process groups: bootstrap and host-staged transport (stdlib only).

Two uses, neither of them on the data path of a real multi-GPU run:
  * bootstrap of the library's RCCL communicator (karma_amd/comm.py RcclComm):
    rank 0's 128-byte unique id reaches the other ranks, and host scalars
    (timings, counts) are gathered;
  * the transport of HostComm, which stages the exchange through host memory
    for rehearsals where RCCL cannot run: several ranks on ONE GPU (RCCL
    refuses duplicate devices), or CPU-only tests of the sharding logic.

SocketGroup is a TCP star on the launcher's rendezvous address (one process
per rank, e.g. under torchrun); ThreadGroup holds the ranks as threads of one
process.  Both expose the same two calls: allgather(ndarray) -> list of every
rank's array, and barrier().
"""

from __future__ import annotations

import os
import socket
import struct
import threading
import time

import numpy as np


def _send_msg(sock, payload: bytes):
    sock.sendall(struct.pack("<Q", len(payload)) + payload)


def _recv_exact(sock, n):
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            raise ConnectionError("host group peer closed the connection")
        got += k
    return bytes(buf)


def _recv_msg(sock) -> bytes:
    (n,) = struct.unpack("<Q", _recv_exact(sock, 8))
    return _recv_exact(sock, n)


def _pack(arr: np.ndarray) -> bytes:
    arr = np.ascontiguousarray(arr).reshape(-1)
    dt = arr.dtype.str.encode()
    return struct.pack("<B", len(dt)) + dt + arr.tobytes()


def _unpack(b: bytes) -> np.ndarray:
    n = b[0]
    dt = np.dtype(b[1:1 + n].decode())
    return np.frombuffer(b[1 + n:], dtype=dt).copy()


_HELLO = b"KRMA"


def _is_local(addr):
    return addr in ("127.0.0.1", "localhost", "::1", "0.0.0.0") or addr == socket.gethostname()


class SocketGroup:
    """TCP star: rank 0 listens on (addr, port), the others connect.

    allgather: every rank sends its array to rank 0, which returns the list of
    all of them to every rank.  Message sizes are whatever the arrays hold.

    Port: `port` is tried first.  When it is taken and `handshake` names a file
    (single-node jobs, from_env), rank 0 listens on a free port instead and
    publishes it there (atomic rename); the other ranks re-read that file on
    every connect attempt.  A connection is accepted only after a 4-byte hello
    both ways, so a stale file or a foreign listener is retried, not trusted.
    Without a handshake file a taken port fails at once, naming
    KARMA_GROUP_PORT.  The other ranks give up after `timeout` seconds."""

    def __init__(self, world, rank, addr="127.0.0.1", port=29600, timeout=120.0, handshake=None):
        self.world, self.rank = world, rank
        self.peers = {}
        self.sock = None
        self.handshake = None
        if world == 1:
            return
        if rank == 0:
            self._serve(addr, port, timeout, handshake)
        else:
            self._connect(addr, port, timeout, handshake)

    def _serve(self, addr, port, timeout, handshake):
        srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        try:
            srv.bind((addr, port))
        except OSError as e:
            if handshake is None:
                srv.close()
                raise OSError(e.errno, f"host group: rank 0 cannot listen on {addr}:{port} ({e.strerror}); "
                                       f"set KARMA_GROUP_PORT to a free port") from e
            srv.bind((addr, 0))
        port = srv.getsockname()[1]
        if handshake is not None:
            tmp = f"{handshake}.{os.getpid()}.tmp"
            with open(tmp, "w") as f:
                f.write(str(port))
            os.replace(tmp, handshake)
            self.handshake = handshake
        srv.listen(self.world)
        srv.settimeout(timeout)
        try:
            while len(self.peers) < self.world - 1:
                c, _ = srv.accept()
                c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                c.settimeout(30.0)
                try:
                    hello = _recv_exact(c, 8)
                except (OSError, ConnectionError):
                    c.close()
                    continue
                if hello[:4] != _HELLO:  # not a karma rank (a stale dialler, a port scan): ignored
                    c.close()
                    continue
                (r,) = struct.unpack("<i", hello[4:])
                if not 0 < r < self.world or r in self.peers:
                    # a karma rank with a rank this job cannot hold: a misconfigured
                    # launch (two processes with one RANK, or WORLD_SIZE disagreeing)
                    c.close()
                    what = "a duplicate" if r in self.peers else f"out of range for world size {self.world}"
                    raise ConnectionError(f"host group: a rank connected as rank {r}, {what}")
                c.sendall(_HELLO)
                c.settimeout(None)
                self.peers[r] = c
        finally:
            srv.close()

    def _connect(self, addr, port, timeout, handshake):
        deadline = time.time() + timeout
        while True:
            p = port
            if handshake is not None:
                try:
                    with open(handshake) as f:
                        p = int(f.read().strip() or port)
                except (OSError, ValueError):
                    pass
            try:
                s = socket.create_connection((addr, p), timeout=5)
                s.settimeout(10.0)
                s.sendall(_HELLO + struct.pack("<i", self.rank))
                if _recv_exact(s, 4) != _HELLO:
                    raise ConnectionError("not a karma host group")
                break
            except (OSError, ConnectionError):
                try:
                    s.close()
                except Exception:
                    pass
                if time.time() > deadline:
                    raise TimeoutError(f"host group: rank {self.rank} could not reach rank 0 at {addr}:{p} within "
                                       f"{timeout:.0f} s (KARMA_GROUP_PORT / KARMA_GROUP_TIMEOUT)")
                time.sleep(0.05)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        s.settimeout(None)
        self.sock = s

    @classmethod
    def from_env(cls, world=None, rank=None):
        """Ranks started by a launcher (torchrun): RANK / WORLD_SIZE / MASTER_ADDR,
        port KARMA_GROUP_PORT, else MASTER_PORT + 1 (torchrun's own store holds
        MASTER_PORT) with a handshake file in the temp directory when the job is
        on this node, so a taken port moves instead of stalling the job."""
        import tempfile

        world = int(os.environ.get("WORLD_SIZE", "1")) if world is None else world
        rank = int(os.environ.get("RANK", "0")) if rank is None else rank
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        timeout = float(os.environ.get("KARMA_GROUP_TIMEOUT", "120"))
        fixed = os.environ.get("KARMA_GROUP_PORT")
        mport = int(os.environ.get("MASTER_PORT", "29500"))
        port = int(fixed) if fixed else mport + 1
        handshake = None
        # the port fallback publishes the new port in a local file: only when
        # every rank runs on this node (a remote rank could not read it)
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        if not fixed and _is_local(addr) and local_world == world:
            run = os.environ.get("TORCHELASTIC_RUN_ID", "none")
            handshake = os.path.join(tempfile.gettempdir(), f"karma_group_{run}_{mport}.port")
        return cls(world, rank, addr, port, timeout=timeout, handshake=handshake)

    def allgather(self, arr) -> list:
        arr = np.asarray(arr)
        if self.world == 1:
            return [np.ascontiguousarray(arr).reshape(-1).copy()]
        if self.rank == 0:
            parts = [None] * self.world
            parts[0] = _pack(arr)
            for r, c in self.peers.items():
                parts[r] = _recv_msg(c)
            blob = struct.pack("<i", self.world) + b"".join(struct.pack("<Q", len(p)) + p for p in parts)
            for c in self.peers.values():
                _send_msg(c, blob)
        else:
            _send_msg(self.sock, _pack(arr))
            blob = _recv_msg(self.sock)
        (w,) = struct.unpack_from("<i", blob, 0)
        out, off = [], 4
        for _ in range(w):
            (n,) = struct.unpack_from("<Q", blob, off)
            off += 8
            out.append(_unpack(blob[off:off + n]))
            off += n
        return out

    def barrier(self):
        self.allgather(np.zeros(0, np.uint8))

    def close(self):
        for c in self.peers.values():
            c.close()
        self.peers = {}
        if self.handshake is not None:
            try:
                os.remove(self.handshake)
            except OSError:
                pass
            self.handshake = None
        if self.sock is not None:
            self.sock.close()
            self.sock = None


class _ThreadState:
    def __init__(self, world):
        self.world = world
        self.barrier = threading.Barrier(world)
        self.slots = [None] * world


class ThreadGroup:
    """Ranks as threads of one process (host-staged multi-rank rehearsal).

    ThreadGroup.create(W) returns the W per-rank handles; each rank's thread
    uses its own handle."""

    def __init__(self, state, rank):
        self.state, self.rank, self.world = state, rank, state.world

    @classmethod
    def create(cls, world):
        st = _ThreadState(world)
        return [cls(st, r) for r in range(world)]

    def allgather(self, arr) -> list:
        st = self.state
        st.slots[self.rank] = np.ascontiguousarray(arr).reshape(-1).copy()
        st.barrier.wait()
        out = list(st.slots)
        st.barrier.wait()  # nobody overwrites a slot before everyone has read it
        return out

    def barrier(self):
        self.state.barrier.wait()

    def close(self):
        pass


def run_ranks(world, fn, *args):
    """Run fn(group, rank, *args) on `world` threads sharing one ThreadGroup;
    returns the per-rank results (re-raises the first failure, after breaking
    the group's barrier so no rank waits forever)."""
    groups = ThreadGroup.create(world)
    results = [None] * world
    errors = [None] * world

    def body(r):
        try:
            results[r] = fn(groups[r], r, *args)
        except BaseException as e:  # noqa: BLE001 (re-raised below)
            errors[r] = e
            groups[r].state.barrier.abort()

    threads = [threading.Thread(target=body, args=(r,), name=f"karma-rank{r}") for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    for e in errors:
        if e is not None and not isinstance(e, threading.BrokenBarrierError):
            raise e
    for e in errors:
        if e is not None:
            raise e
    return results

"""Torch-free rank rendezvous for the multi-process benchmark: rank 0 listens on a TCP port
of MASTER_ADDR, every other rank connects once, and the open connections carry the three
host-side collectives the run needs -- the RCCL unique-id broadcast before the
communicator exists, a barrier, and the max over ranks of the step time.

The device data path never goes through here (the halo moves over RCCL, csrc/mpas_halo.hip);
this replaces the torch.distributed process group bench.py used in round 2, whose import
put torch's bundled HIP runtime into the process beside the one libmpasdyn links
(INTEGRATION.md "One HIP runtime per process").

Port: MPAS_RDZV_PORT when set (bench.py's own launcher picks a free one), else
MASTER_PORT + 1 (under torch.distributed.run MASTER_PORT is the launcher's store).
"""
import os
import socket
import struct
import time


def rdzv_port(env=None):
    env = os.environ if env is None else env
    if "MPAS_RDZV_PORT" in env:
        return int(env["MPAS_RDZV_PORT"])
    return int(env["MASTER_PORT"]) + 1


def _send(s, b):
    s.sendall(struct.pack("!I", len(b)) + b)


def _recv_exact(s, n):
    buf = bytearray()
    while len(buf) < n:
        chunk = s.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("rendezvous peer closed the connection")
        buf += chunk
    return bytes(buf)


def _recv(s):
    (n,) = struct.unpack("!I", _recv_exact(s, 4))
    return _recv_exact(s, n)


class Rendezvous:
    """world ranks on one node; rank 0 is the hub.  Every call is collective (all ranks
    call it in the same order)."""

    def __init__(self, rank, world, addr="127.0.0.1", port=None, timeout=300.0):
        self.rank, self.world = int(rank), int(world)
        port = rdzv_port() if port is None else int(port)
        self.peers = []  # rank 0: the sockets of ranks 1..world-1, in rank order
        self.hub = None  # rank > 0: the socket to rank 0
        if self.world == 1:
            return
        deadline = time.monotonic() + timeout
        if self.rank == 0:
            ls = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            ls.bind((addr, port))
            ls.listen(self.world)
            ls.settimeout(timeout)
            got = {}
            try:
                while len(got) < self.world - 1:
                    c, _ = ls.accept()
                    c.settimeout(timeout)
                    (r,) = struct.unpack("!I", _recv(c))
                    if not 0 < r < self.world or r in got:
                        raise ConnectionError(f"rendezvous: unexpected rank {r}")
                    got[r] = c
            finally:
                ls.close()
            self.peers = [got[r] for r in range(1, self.world)]
        else:
            while True:
                try:
                    s = socket.create_connection((addr, port), timeout=5.0)
                    break
                except OSError:
                    if time.monotonic() > deadline:
                        raise
                    time.sleep(0.05)
            s.settimeout(timeout)
            _send(s, struct.pack("!I", self.rank))
            self.hub = s

    def bcast(self, data=None):
        """rank 0's bytes on every rank"""
        if self.world == 1:
            return bytes(data)
        if self.rank == 0:
            for s in self.peers:
                _send(s, bytes(data))
            return bytes(data)
        return _recv(self.hub)

    def allreduce_max(self, x):
        """max over ranks of a float, on every rank"""
        if self.world == 1:
            return float(x)
        if self.rank == 0:
            m = float(x)
            for s in self.peers:
                m = max(m, struct.unpack("!d", _recv(s))[0])
            for s in self.peers:
                _send(s, struct.pack("!d", m))
            return m
        _send(self.hub, struct.pack("!d", float(x)))
        return struct.unpack("!d", _recv(self.hub))[0]

    def barrier(self):
        self.allreduce_max(0.0)

    def close(self):
        for s in self.peers + ([self.hub] if self.hub else []):
            try:
                s.close()
            except OSError:
                pass
        self.peers, self.hub = [], None

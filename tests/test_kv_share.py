"""disagg/kv_share.py's fd hand-over (CPU): the owner serves a list of fds on
an abstract Unix socket (SCM_RIGHTS), a peer receives duplicates of exactly
those, in order, in batches past the per-message limit.  The VMM allocation
and mapping around it run on the GPU (tools/ipc_probe.py --vmm-gib,
profiles/r6_ipc_probe_vmm.json; tests/test_disagg_loopback.py two-process
bench)."""
import os

from dynamo_exp_amd.disagg import kv_share


class _FakeBuf(kv_share.SharedKVBuffer):
    """SharedKVBuffer's serving half over ordinary pipe fds (no device)."""

    def __init__(self, fds, chunk):
        self._fds = None
        self._sock = None
        self.address = None
        self._closed = False
        self.chunk = chunk
        self.total = chunk * len(fds)
        self._pipe_fds = fds

        class _K:
            @staticmethod
            def vmm_export_fds(handles):
                return list(fds)

        self._k = _K()
        self._handles = []


def test_fds_handed_over_in_order_cpu():
    pipes = [os.pipe() for _ in range(kv_share._MAX_FDS + 7)]  # two messages
    buf = _FakeBuf([w for _, w in pipes], 1 << 20)
    addr = buf.serve("test")
    fds, chunk, total = kv_share._recv_fds(addr)
    try:
        assert chunk == 1 << 20 and total == chunk * len(pipes) and len(fds) == len(pipes)
        for i, ((r, _), fd) in enumerate(zip(pipes, fds)):
            os.write(fd, bytes([i % 256]))  # the received fd is the same pipe's write end
            assert os.read(r, 1) == bytes([i % 256])
    finally:
        buf._closed = True
        buf._sock.close()
        for fd in fds:
            os.close(fd)
        for r, w in pipes:
            os.close(r)
            os.close(w)


def test_recv_fails_cleanly_without_owner_cpu():
    import pytest

    with pytest.raises(OSError):
        kv_share._recv_fds(b"\0dx-kvshare-nobody".hex(), timeout=2.0)


def test_chunk_sizing_cpu():
    MiB, GiB = 1 << 20, 1 << 30
    assert kv_share.chunk_for(6 * GiB) == 512 * MiB  # small caches: the default chunk
    assert kv_share.chunk_for(240 * GiB) == -(-240 * GiB // 256)  # <= 256 fds
    assert kv_share.chunk_for(288 * GiB) == GiB  # never above 1 GiB per allocation

"""Process-group rendezvous for one process per GPU on one node, without
torch and without touching the GPU.

A rank launched by `torchrun --nnodes=1` (RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT in the environment) needs a side channel for three small things:
rank 0's RCCL unique id (so every rank can join the library's RCCL
communicator, bm_ctx_create_rank), barriers around a timed region, and a max
over ranks of the elapsed time.  The data path does not go through here: the
per-rank 16-byte partials are combined by the library's RCCL allgather.

Why not torch.distributed: importing torch maps torch's own HIP runtime, and
on this image it opens the GPU (a gloo sidecar per rank doubled the processes
holding the GPU: 8 ranks + 8 sidecars + the launcher exceeded the box's
16-process guard).  The ranks of one node share a filesystem, so each
collective is a set of small files: rank r writes `<seq>.<r>` (atomically,
by rename) and every rank waits until all `world` files of that step exist.
The directory is keyed by MASTER_ADDR, MASTER_PORT, the launcher's pid (all
ranks of one torchrun launch share their parent) and torchrun's run id and
restart count (an elastic restart keeps the same parent: its ranks must not
meet the failed attempt's files), and rank 0 removes it once every rank has
left.

`all_gather` also carries the partials for the one-GPU rehearsal (every rank
on device 0, where RCCL cannot place two ranks on one GPU) and for CPU tests.
"""
import json
import os
import shutil
import tempfile
import time


class Rendezvous:
    """The calling process's seat in the group of one node's ranks."""

    def __init__(self, timeout_s: float = 600.0, path: str = None):
        self.rank = int(os.environ["RANK"])
        self.world = int(os.environ["WORLD_SIZE"])
        self.timeout_s = timeout_s
        key = "-".join([os.environ.get("MASTER_ADDR", "local"), os.environ.get("MASTER_PORT", "0"), str(os.getppid()),
                        os.environ.get("TORCHELASTIC_RUN_ID", "none"),
                        os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")])
        key = "".join(ch if ch.isalnum() or ch in "-_." else "_" for ch in key)
        self.path = path or os.environ.get("BTCMINER_RDZV_DIR") or os.path.join(
            tempfile.gettempdir(), f"btcminer-rdzv-{key}")
        os.makedirs(self.path, exist_ok=True)
        self._seq = 0
        self._open = True
        self.barrier()

    def _wait(self, names):
        deadline = time.monotonic() + self.timeout_s
        pause = 5e-5
        while True:
            if all(os.path.exists(n) for n in names):
                return
            if time.monotonic() > deadline:
                missing = [os.path.basename(n) for n in names if not os.path.exists(n)]
                raise RuntimeError(f"rendezvous {self.path}: rank {self.rank} timed out waiting for {missing}")
            time.sleep(pause)
            pause = min(pause * 2, 1e-3)

    def _post(self, name, obj):
        tmp = os.path.join(self.path, f".{name}.tmp")
        with open(tmp, "w") as f:
            json.dump(obj, f)
        os.replace(tmp, os.path.join(self.path, name))

    def all_gather(self, obj):
        """List of every rank's JSON-able obj, by rank."""
        if not self._open:
            raise RuntimeError("rendezvous closed")
        seq = self._seq
        self._seq += 1
        self._post(f"{seq}.{self.rank}", obj)
        names = [os.path.join(self.path, f"{seq}.{r}") for r in range(self.world)]
        self._wait(names)
        out = []
        for n in names:
            with open(n) as f:
                out.append(json.load(f))
        return out

    def broadcast_bytes(self, data: bytes = None, src: int = 0) -> bytes:
        """src's bytes on every rank."""
        return bytes.fromhex(self.all_gather(data.hex() if self.rank == src else None)[src])

    def barrier(self):
        self.all_gather(None)

    def all_max(self, x: float) -> float:
        return max(self.all_gather(float(x)))

    def close(self):
        if not self._open:
            return
        self.barrier()
        self._open = False
        self._post(f"left.{self.rank}", None)
        if self.rank == 0:  # every rank has passed the last barrier and said so
            self._wait([os.path.join(self.path, f"left.{r}") for r in range(self.world)])
            shutil.rmtree(self.path, ignore_errors=True)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

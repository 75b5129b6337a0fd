"""Process-group rendezvous for one process per GPU, kept out of the GPU
process.

A rank of `torchrun` (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the
environment) needs a side channel for three small things: rank 0's RCCL
unique id (so every rank can join the library's RCCL communicator,
bm_ctx_create_rank), barriers around a timed region, and a max over ranks of
the elapsed time.  torch.distributed's gloo backend provides them, but
importing torch maps torch's bundled HIP runtime next to the /opt/rocm one
libbtcminer.so uses.  So torch runs in a sidecar child process that joins the
gloo group as this rank and serves requests over a pipe (one JSON line each
way); the GPU process itself never imports torch.

The data path does not go through here: the per-rank 16-byte partials are
combined by the library's own RCCL allgather.  `all_gather` exists for the
one-GPU rehearsal (every rank on device 0, where RCCL cannot place two ranks
on one GPU) and for CPU tests.
"""
import json
import os
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))


class Rendezvous:
    """The calling process's seat in the torchrun group (env://, gloo)."""

    def __init__(self, timeout_s: float = 600.0):
        self.rank = int(os.environ["RANK"])
        self.world = int(os.environ["WORLD_SIZE"])
        env = dict(os.environ)
        env["PYTHONPATH"] = os.path.dirname(_HERE) + os.pathsep + env.get("PYTHONPATH", "")
        self._p = subprocess.Popen([sys.executable, "-u", "-m", "distributed_bitcoin_minter_amd.rendezvous",
                                    str(timeout_s)], stdin=subprocess.PIPE, stdout=subprocess.PIPE, env=env,
                                   text=True, bufsize=1)
        self._call("ready")

    def _call(self, op, value=None):
        self._p.stdin.write(json.dumps({"op": op, "value": value}) + "\n")
        self._p.stdin.flush()
        line = self._p.stdout.readline()
        if not line:
            raise RuntimeError(f"rendezvous sidecar of rank {self.rank} exited (code {self._p.poll()})")
        out = json.loads(line)
        if "error" in out:
            raise RuntimeError(f"rendezvous {op}: {out['error']}")
        return out.get("value")

    def broadcast_bytes(self, data: bytes = None, src: int = 0) -> bytes:
        """src's bytes on every rank."""
        return bytes.fromhex(self._call("bcast", data.hex() if self.rank == src else None))

    def barrier(self):
        self._call("barrier")

    def all_max(self, x: float) -> float:
        return self._call("max", float(x))

    def all_gather(self, obj):
        """List of every rank's JSON-able obj, by rank."""
        return self._call("gather", obj)

    def close(self):
        if self._p is None:
            return
        try:
            self._call("close")
        except (RuntimeError, OSError, ValueError):
            pass
        try:
            self._p.wait(timeout=60)
        except subprocess.TimeoutExpired:
            self._p.kill()
            self._p.wait()
        self._p = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def _serve(timeout_s: float):
    """Sidecar: join the gloo group as $RANK and answer requests on stdin."""
    # replies go to the original stdout; anything torch / gloo print (gloo
    # logs "[Gloo] Rank 0 is connected ..." to stdout) goes to stderr
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    sys.stdout = sys.stderr
    import datetime
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=timeout_s))
    rank, world = dist.get_rank(), dist.get_world_size()
    for line in sys.stdin:
        req = json.loads(line)
        op, value = req["op"], req.get("value")
        try:
            if op == "ready":
                res = None
            elif op == "bcast":
                box = [value]
                dist.broadcast_object_list(box, src=0)
                res = box[0]
            elif op == "barrier":
                dist.barrier()
                res = None
            elif op == "max":
                t = torch.tensor([value], dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                res = t.item()
            elif op == "gather":
                box = [None] * world
                dist.all_gather_object(box, value)
                res = box
            elif op == "close":
                out.write(json.dumps({"value": None}) + "\n")
                out.flush()
                break
            else:
                raise ValueError(f"unknown op {op!r}")
            out.write(json.dumps({"value": res}) + "\n")
        except Exception as e:  # report to the GPU process, which raises
            out.write(json.dumps({"error": f"rank {rank}: {e!r}"}) + "\n")
        out.flush()
    dist.destroy_process_group()


if __name__ == "__main__":
    _serve(float(sys.argv[1]) if len(sys.argv) > 1 else 600.0)

"""Control plane of the N>1 bench: barrier and all-gather among the ranks of
one node, through files, with no torch import.

The data path has no collective (independent packet shards,
per-GPU map shards merged on the host), so the ranks only need to agree on
when the timed region starts and ends and to hand rank 0 their timings and
map shards.  `torch.distributed` would do that, but importing torch loads
its bundled HIP runtime (libamdhip64.so.7 of ROCm 7.0, the same SONAME as
/opt/rocm's 7.2), so the interpreter kernel would run on a different runtime
at N>1 than at N=1.  This module keeps every rank count on the library's own
runtime.

Ranks meet in a directory under /tmp named after the launch: torchrun's
elastic agent is the parent of every worker of one launch, so its pid and
start time (from /proc), MASTER_PORT and the agent's run id
(TORCHELASTIC_RUN_ID) identify the launch, with the user's uid; a later
launch never sees an earlier one's files.  `BPFTIME_AMD_RDZV_DIR` names the
directory instead; ranks started outside torchrun must name one (their
parent, a shell, would give every run from it the same directory).  The
directory is made 0700 and refused when it is not a directory of this user
that only this user can write, or when it holds a finished launch's files
(a predictable /tmp path another user could plant).  Each message is a file written under a temporary name
and renamed into place (atomic on one filesystem); waiting is polling with
a sleep that grows to 1 ms.
"""
from __future__ import annotations

import base64
import json
import os
import shutil
import time
from typing import Any, List, Optional


def _proc_start(pid: int) -> str:
    try:
        with open(f"/proc/{pid}/stat") as f:
            stat = f.read()
        return stat.rsplit(")", 1)[1].split()[19]  # field 22: starttime
    except (OSError, IndexError):
        return "0"


def launch_dir() -> str:
    d = os.environ.get("BPFTIME_AMD_RDZV_DIR")
    if d:
        return d
    run = os.environ.get("TORCHELASTIC_RUN_ID")
    if run is None:
        raise RuntimeError("ranks started outside torchrun need BPFTIME_AMD_RDZV_DIR (a directory for this launch)")
    run = "".join(c if c.isalnum() or c in "-_" else "_" for c in run)[:64]
    ppid = os.getppid()
    port = os.environ.get("MASTER_PORT", "0")
    return os.path.join("/tmp", f"bpftime_amd_rdzv_{os.getuid()}_{ppid}_{_proc_start(ppid)}_{port}_{run}")


def _check_dir(path: str) -> None:
    import stat
    st = os.lstat(path)
    if not stat.S_ISDIR(st.st_mode) or st.st_uid != os.getuid() or st.st_mode & 0o077:
        raise PermissionError(f"refusing rendezvous directory {path}: it must be a directory of uid {os.getuid()} "
                              f"with mode 0700 (found uid {st.st_uid}, mode {oct(st.st_mode & 0o7777)})")


def _enc(obj: Any) -> Any:
    if isinstance(obj, (bytes, bytearray)):
        return {"__b64__": base64.b64encode(bytes(obj)).decode()}
    if isinstance(obj, (list, tuple)):
        return [_enc(x) for x in obj]
    if isinstance(obj, dict):
        return {k: _enc(v) for k, v in obj.items()}
    return obj


def _dec(obj: Any) -> Any:
    if isinstance(obj, dict):
        if set(obj) == {"__b64__"}:
            return base64.b64decode(obj["__b64__"])
        return {k: _dec(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_dec(x) for x in obj]
    return obj


class Rendezvous:
    """Barrier / all-gather among `world` ranks of one node."""

    def __init__(self, rank: int, world: int, path: Optional[str] = None, timeout: float = 600.0):
        self.rank, self.world, self.timeout = rank, world, timeout
        self.path = path or launch_dir()
        self.seq = 0
        os.makedirs(self.path, mode=0o700, exist_ok=True)
        _check_dir(self.path)
        if rank == 0 and any(n.startswith("exit.") for n in os.listdir(self.path)):
            raise RuntimeError(f"rendezvous directory {self.path} holds a finished launch's files")

    def _put(self, name: str, data: bytes) -> None:
        tmp = os.path.join(self.path, f".{name}.{self.rank}.tmp")
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, os.path.join(self.path, name))

    def _wait(self, names: List[str]) -> None:
        t0, nap = time.monotonic(), 50e-6
        pending = list(names)
        while pending:
            pending = [n for n in pending if not os.path.exists(os.path.join(self.path, n))]
            if not pending:
                return
            if time.monotonic() - t0 > self.timeout:
                raise TimeoutError(f"rendezvous {self.path}: rank {self.rank} waited {self.timeout:.0f} s "
                                   f"for {pending[:4]}")
            time.sleep(nap)
            nap = min(nap * 2, 1e-3)

    def barrier(self) -> None:
        self.seq += 1
        self._put(f"b{self.seq}.{self.rank}", b"")
        self._wait([f"b{self.seq}.{r}" for r in range(self.world)])

    def all_gather(self, obj: Any) -> List[Any]:
        """Every rank's obj (JSON values, bytes allowed inside lists / dicts /
        tuples; tuples come back as lists), in rank order, on every rank."""
        self.seq += 1
        self._put(f"g{self.seq}.{self.rank}", json.dumps(_enc(obj)).encode())
        names = [f"g{self.seq}.{r}" for r in range(self.world)]
        self._wait(names)
        out = []
        for n in names:
            with open(os.path.join(self.path, n), "rb") as f:
                out.append(_dec(json.loads(f.read())))
        return out

    def close(self) -> None:
        """A last barrier; every other rank then says it has left it, and
        rank 0 removes the directory once all have (a rank still polling
        the barrier must not find its files gone)."""
        self.barrier()
        if self.rank != 0:
            self._put(f"exit.{self.rank}", b"")
            return
        self._wait([f"exit.{r}" for r in range(1, self.world)])
        shutil.rmtree(self.path, ignore_errors=True)

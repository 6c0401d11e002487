"""Single-node rank launcher: ``python bench.py --gpus N`` starts N ranks itself.

The parent process never touches the GPU (no torch import, no HIP call): it
picks a free rendezvous port on 127.0.0.1, starts N fresh child interpreters
running the same script with ``RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT`` set (the variables ``torch.distributed.run`` would set), forwards
their output, and exits with the first non-zero child status (the remaining
ranks are then terminated, so a crashed rank cannot leave the others blocked in
a collective).  Children are started with ``subprocess`` -- never ``exec`` --
so nothing replaces a process that has initialised a device.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional, Sequence


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket() as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def launched_by_launcher() -> bool:
    """True inside a rank started by torchrun or by :func:`spawn_ranks`."""
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def spawn_ranks(n: int, argv: Optional[Sequence[str]] = None, env: Optional[dict] = None,
                poll_s: float = 0.2) -> int:
    """Run ``python <argv>`` as ``n`` ranks of one process group; returns the exit
    status (0 when every rank succeeded)."""
    argv = list(sys.argv if argv is None else argv)
    base = dict(os.environ if env is None else env)
    base.setdefault("MASTER_ADDR", "127.0.0.1")
    base["MASTER_PORT"] = str(free_port(base["MASTER_ADDR"]))
    base["WORLD_SIZE"] = str(n)
    base["LOCAL_WORLD_SIZE"] = str(n)
    base.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 8) // max(n, 1))))
    procs: List[subprocess.Popen] = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), GROUP_RANK="0")
        procs.append(subprocess.Popen([sys.executable, "-u"] + argv, env=e, start_new_session=True))
    status = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                status = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(poll_s)
    except KeyboardInterrupt:
        status = 130
    finally:
        if status != 0:
            for p in procs:
                if p.poll() is None:
                    try:
                        os.killpg(p.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
            deadline = time.time() + 10
            for p in procs:
                try:
                    p.wait(timeout=max(0.1, deadline - time.time()))
                except subprocess.TimeoutExpired:
                    try:
                        os.killpg(p.pid, signal.SIGKILL)
                    except ProcessLookupError:
                        pass
                    p.wait()
    if status < 0:               # killed by a signal: report it like a shell does
        status = 128 - status
    return int(status)

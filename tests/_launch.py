"""Start a world of gloo ranks running tests/_dist_worker.py and collect their verdicts."""

import json
import os
import socket
import subprocess
import sys
import tempfile
from pathlib import Path

WORKER = Path(__file__).resolve().parent / "_dist_worker.py"


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_world(mode: str, world: int, timeout: int, extra_env=None):
    port = free_port()
    with tempfile.TemporaryDirectory() as d:
        procs, outs = [], []
        for r in range(world):
            env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="2")
            env.update(extra_env or {})
            out = Path(d) / f"rank{r}.json"
            outs.append(out)
            procs.append(subprocess.Popen([sys.executable, str(WORKER), mode, str(out)], env=env,
                                          stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
        logs = []
        try:
            for p in procs:
                logs.append(p.communicate(timeout=timeout)[0].decode(errors="replace"))
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
                    p.wait()
        res = []
        for r, out in enumerate(outs):
            if not out.exists():
                res.append({"ok": False, "why": f"rank {r} wrote no verdict (rc {procs[r].returncode}):\n{logs[r][-3000:]}"})
            else:
                res.append(json.loads(out.read_text()))
        return res

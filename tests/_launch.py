"""Start a world of gloo ranks running tests/_dist_worker.py and collect their verdicts.

While the ranks run, a line is appended every 20 s to the file named by EON_TEST_HEARTBEAT (if
set; tools/gpu_tests.sh points it under gpurun_out/), so a long multi-rank test is not mistaken for
a hung command."""

import json
import os
import socket
import subprocess
import sys
import tempfile
import time
from pathlib import Path

WORKER = Path(__file__).resolve().parent / "_dist_worker.py"


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _heartbeat(msg: str):
    hb = os.environ.get("EON_TEST_HEARTBEAT")
    if hb:
        with open(hb, "a") as f:
            f.write(f"{time.strftime('%H:%M:%S')} {msg}\n")


def run_world(mode: str, world: int, timeout: int, extra_env=None):
    port = free_port()
    with tempfile.TemporaryDirectory() as d:
        procs, outs, logs = [], [], []
        for r in range(world):
            env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="2")
            env.update(extra_env or {})
            out = Path(d) / f"rank{r}.json"
            outs.append(out)
            log = open(Path(d) / f"rank{r}.log", "wb")
            logs.append(log)
            procs.append(subprocess.Popen([sys.executable, str(WORKER), mode, str(out)], env=env,
                                          stdout=log, stderr=subprocess.STDOUT))
        t0 = last = time.monotonic()
        try:
            while any(p.poll() is None for p in procs):
                now = time.monotonic()
                if now - t0 > timeout:
                    break
                if now - last >= 20:
                    _heartbeat(f"run_world {mode} x{world}: {now - t0:.0f} s, "
                               f"{sum(p.poll() is None for p in procs)} ranks running")
                    last = now
                time.sleep(0.5)
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
                    p.wait()
            for f in logs:
                f.close()
        res = []
        for r, out in enumerate(outs):
            if not out.exists():
                text = (Path(d) / f"rank{r}.log").read_bytes().decode(errors="replace")
                res.append({"ok": False, "why": f"rank {r} wrote no verdict (rc {procs[r].returncode}):\n{text[-3000:]}"})
            else:
                res.append(json.loads(out.read_text()))
        return res

"""RCCL on hardware: the result exchange bench.py times at N > 1 -- the "nccl" process
group bound to the device, the weight broadcast, the packed all_gather in its blocking and overlapped
forms -- run over a real RCCL communicator (world size 1: the box has one GPU, and RCCL takes one rank
per device).  In a child process, so the communicator's lifetime ends with it; the gloo world-size-2
test (test_distributed_cpu.py) covers the multi-rank sharding itself."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_world1_gather_equals_local():
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "rccl_world1.py"), str(_free_port())],
                       capture_output=True, text=True, timeout=100, cwd=ROOT)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["backend"] == "nccl" and line["checked"] == ["visits", "action", "root_q"], line

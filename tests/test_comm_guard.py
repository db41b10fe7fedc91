"""CPU failure injection for the collective abort protocol of the RCCL
transport (tsne-flink_amd/csrc/comm_guard.hpp, used by comm.cpp RcclComm):
a rank waiting in a collective whose peer died is released by abort() from
the peer's thread (no lock is held across a wait: the round-4 advisor's
deadlock), and nothing reaches the communicator after abort freed it (the
round-3 advisor's use-after-free).  A fake backend stands in for RCCL."""
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def test_comm_guard_abort_protocol(tmp_path):
    exe = tmp_path / "comm_guard_test"
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-pthread", "-I", str(ROOT / "tsne-flink_amd" / "csrc"),
                           str(ROOT / "tests" / "native" / "comm_guard_test.cpp"), "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout + out.stderr

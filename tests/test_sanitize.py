"""Host-side sanitizers: tools/sanitize_host.sh builds the Node-API addon, a CPU
stand-in of the C ABI, the host build of the device arithmetic and the oracle's C port with
-fsanitize=address,undefined and runs them (addon entry points, pass slots, close() with passes in
flight, GC finalisation, the JS verifier's CPU suite, tests/test_host_arith.py, tests/test_cpu_port.py).
Any sanitizer report aborts the run."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("node") is None or not os.path.exists("/usr/include/node/node_api.h"),
                    reason="node / node_api.h not installed")
def test_host_code_is_sanitizer_clean(tmp_path):
    p = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize_host.sh"), str(tmp_path)], capture_output=True, text=True,
                       timeout=600)
    assert p.returncode == 0 and "[sanitize] clean" in p.stdout, (p.stdout[-3000:], p.stderr[-6000:])
    r = json.load(open(tmp_path / "addon_stub.json"))
    assert "fatal" not in r, r
    assert all(v is True for k, v in r.items() if isinstance(v, bool)), r
    assert r["streamed"] == [True, True, True] and r["busyThrows"] == "GBV_E_BUSY" and r["waitTwice"] == "GBV_E_ARG"
    assert r["afterClose"] == "QUEUE_ABORTED,QUEUE_ABORTED,QUEUE_ABORTED" and r["pendingAtClose"] == "resolved"
    assert r["jsPacked"] is True and r["jsPackedBadLength"] == "GBV_E_ARG"
    v = json.load(open(tmp_path / "verifier_cpu.json"))
    assert "fatal" not in v and v["close"] is True and v["basic"] == [True, False, False], v

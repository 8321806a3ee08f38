"""The Node-API addon in C (addon/gbv_addon.c), the north_star boundary: "a thin Node-API C-ABI
addon, written in C and called from TypeScript" (BASELINE.json).  Built here against
/usr/include/node/node_api.h and loaded by the installed Node (v12), which calls it from JavaScript
(addon/test_addon.js) the way a Lodestar GpuBlsVerifier would (bls/interface.ts:25-68).

CPU: exports, argument errors (TypeError, code GBV_E_ARG) and device errors (GBV_E_DEVICE) -- no GPU.
GPU: every golden case through the addon: verifySets / verifySetsMulti / verifySameMessageMulti,
aggregatePubkeys (byte-exact), EMPTY_AGGREGATE_ARRAY rejection, concurrent calls, close() semantics.
"""
import json
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
ADDON = os.path.join(ROOT, "addon")
NODE = shutil.which("node") or shutil.which("nodejs")

pytestmark = pytest.mark.skipif(NODE is None or not os.path.exists("/usr/include/node/node_api.h"),
                                reason="node / node_api.h not installed")


def _build():
    lib = os.path.join(ROOT, "lodestar_amd", "libgbv.so")
    out = os.path.join(ADDON, "gbv_addon.node")
    src = os.path.join(ADDON, "gbv_addon.c")
    if not os.path.exists(lib):
        from lodestar_amd.build import build
        build()
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(src), os.path.getmtime(lib)):
        subprocess.check_call(["sh", os.path.join(ADDON, "build.sh")])
    return out


def _run(*args, timeout=120):
    _build()
    p = subprocess.run([NODE, os.path.join(ADDON, "test_addon.js")] + list(args), capture_output=True, text=True, timeout=timeout)
    assert p.stdout.strip(), p.stderr
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_addon_builds_and_maps_errors_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("this case checks the no-device error path")
    r = _run("cpu")
    assert r["exports"] == ["open", "addPubkeys", "verifySets", "verifySetsMulti", "verifySameMessageMulti", "aggregatePubkeys",
                            "aggregateSerializedPubkeys", "aggregateSignatures", "validateSignatures", "close"]
    assert r["open"] == "ok"      # gbv_init without a device -> Error code GBV_E_DEVICE
    assert r["badCtx"] == "ok"    # not a context -> TypeError code GBV_E_ARG
    assert r["badArg"] == "ok"


@pytest.mark.gpu
def test_addon_golden_cases_on_gpu():
    r = _run("gpu", os.path.join(HERE, "golden", "fixtures.json"), timeout=300)
    assert "fatal" not in r, r
    assert r["ingest"] is True
    assert all(r["verifySets"]) and len(r["verifySets"]) == 16
    assert all(r["verifySetsMulti"]) and len(r["verifySetsMulti"]) == 16
    assert all(r["sameMessage"]) and r["sameMessage"]
    assert all(r["aggregate"]) and all(r["aggregateSerialized"])
    assert r["emptyAggregate"] == "ok"
    assert all(r["singleThread"]) and len(r["singleThread"]) == 11   # singleThread.ts semantics, incl. swapped_keys
    assert all(r["aggregateSignatures"]) and len(r["aggregateSignatures"]) == 7
    assert r["concurrent"] is True
    assert r["inflightBeforeClose"] is True
    assert r["afterClose"] == "QUEUE_ABORTED"

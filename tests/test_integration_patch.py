"""integration/lodestar-gpu-bls.patch (made by integration/make_patch.py) applies cleanly to the reference
checkout with `patch -p1`: every hunk lands on the files it names.  Needs /root/reference (the build
container); skipped elsewhere.  The TypeScript is not compiled here (no tsc / Node >= 20)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
PATCH = os.path.join(ROOT, "integration", "lodestar-gpu-bls.patch")


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "packages")) or shutil.which("patch") is None,
                    reason="reference checkout / patch(1) not available")
def test_patch_applies_to_reference(tmp_path):
    text = open(PATCH).read()
    files = sorted({l[6:].strip() for l in text.splitlines() if l.startswith("+++ b/")})
    assert len(files) >= 20 and "packages/beacon-node/src/chain/bls/gpu/index.ts" in files
    for rel in files:  # a scratch copy of just the touched files
        src = os.path.join(REF, rel)
        if os.path.exists(src):
            os.makedirs(os.path.dirname(tmp_path / rel), exist_ok=True)
            shutil.copyfile(src, tmp_path / rel)
    p = subprocess.run(["patch", "-p1", "--forward", "--no-backup-if-mismatch", "-i", PATCH], cwd=tmp_path, capture_output=True, text=True)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "FAILED" not in p.stdout and "offset" not in p.stdout, p.stdout
    gpu = (tmp_path / "packages/beacon-node/src/chain/bls/gpu/index.ts").read_text()
    assert "class GpuBlsVerifier implements IBlsVerifier" in gpu
    chain = (tmp_path / "packages/beacon-node/src/chain/chain.ts").read_text()
    assert "opts.blsVerifyOnGpu" in chain and "loadIndex2pubkey" in chain


def _added_file(text, rel):
    """The lines of a file the patch adds (its hunk against /dev/null-style empty a/ side)."""
    out, on = [], False
    for l in text.splitlines():
        if l.startswith("+++ b/"):
            on = l[6:].strip() == rel
            continue
        if on and l.startswith("diff "):
            break
        if on and l.startswith("+"):
            out.append(l[1:])
    return "\n".join(out)


def test_gpu_binding_loads_native_code_lazily():
    """chain/bls/index.ts re-exports GpuBlsVerifier and packages/beacon-node is an ES module
    ("type": "module"): the binding must not `require` at module top level (undefined in ESM, and a
    missing .node file would break every node importing chain/bls).  The addon and the queue load in
    the constructor through createRequire(import.meta.url); the same-message call uses the packed
    form; the node's metric families go to the queue."""
    gpu = _added_file(open(PATCH).read(), "packages/beacon-node/src/chain/bls/gpu/index.ts")
    assert "class GpuBlsVerifier implements IBlsVerifier" in gpu
    top, depth = [], 0
    for line in gpu.splitlines():  # statements at brace depth 0 (module scope)
        if depth == 0:
            top.append(line)
        depth += line.count("{") - line.count("}")
    assert not any("require(" in l for l in top), [l for l in top if "require(" in l]
    ctor = gpu[gpu.index("  constructor("):gpu.index("  loadIndex2pubkey(")]
    assert "createRequire(import.meta.url)" in ctor and 'require("./gbv_addon.node")' in ctor
    assert "nodeMetricFamilies(modules.metrics)" in ctor
    assert "this.queue.verifySameMessageSets(sets, message, opts)" in gpu

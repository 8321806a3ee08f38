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
    assert len(files) >= 15 and "packages/beacon-node/src/chain/bls/gpu/index.ts" in files
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


def test_patch_leaves_callers_alone():
    """north_star: GpuBlsVerifier swaps in "without touching callers".  The patch edits no caller of
    IBlsVerifier -- no file of chain/validation/ outside the signatureSets/ builders, not the interface
    itself -- and the same-message call keeps the interface's {publicKey, signature} shape
    (bls/interface.ts:55-59, validation/attestation.ts:134-137), the key's index found by identity."""
    text = open(PATCH).read()
    files = sorted({l[6:].strip() for l in text.splitlines() if l.startswith("+++ b/")})
    val = "packages/beacon-node/src/chain/validation/"
    callers = [f for f in files if f.startswith(val) and not f.startswith(val + "signatureSets/")]
    assert callers == [], callers
    assert "packages/beacon-node/src/chain/bls/interface.ts" not in files
    gpu = _added_file(text, "packages/beacon-node/src/chain/bls/gpu/index.ts")
    assert "sets: {publicKey: PublicKey; signature: Uint8Array}[]," in gpu and "index?: number" not in gpu
    assert "registerPubkeyObjects" in gpu and "queue.indexOf(set.pubkey)" in gpu and "queue.indicesOf(set.pubkeys)" in gpu

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

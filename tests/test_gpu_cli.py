"""GPU: the kzg_cli driver (kzg-commitments_amd/tools/kzg_cli.cpp), the
counterpart of the reference's demo/shared/kzg-cli.cpp:28-109: setup ->
commit -> prove -> verify through the setup file, the reference's stdout
formats and exit codes (0 valid, 1 invalid)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "kzg-commitments_amd", "tools", "kzg_cli")


def run(*args, cwd):
    return subprocess.run([CLI, *args], cwd=cwd, capture_output=True, text=True, timeout=300)


@pytest.mark.parametrize("curve", ["0", "1"])
def test_cli_round_trip(tmp_path, curve):
    assert os.path.exists(CLI), "run __graft_entry__.build() first"
    setup = str(tmp_path / "kzg_public")
    r = run("--curve", curve, "--setup", setup, "setup", "200", cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    assert "num_coeff=200" in r.stdout and os.path.getsize(setup) > 8
    data = bytes((i * 37 + 11) % 256 for i in range(31 * 20 + 5))
    f = tmp_path / "data.bin"
    f.write_bytes(data)
    r = run("--curve", curve, "--setup", setup, "commit", str(f), cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    commit = r.stdout.strip()
    mb = 32 if curve == "0" else 48
    assert len(commit) == 2 * (4 + 1 + 2 * mb)
    r = run("--curve", curve, "--setup", setup, "prove", str(f), "7", cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    proof, chunk, sub = r.stdout.split()
    assert int(chunk) == 7 % (len(data) // (mb - 1) - 4)
    r = run("--curve", curve, "--setup", setup, "verify", commit, proof, chunk, sub, cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    bad = ("0" if sub[0] != "0" else "1") + sub[1:]
    r = run("--curve", curve, "--setup", setup, "verify", commit, proof, chunk, bad, cwd=tmp_path)
    assert r.returncode == 1, r.stderr
    r = run("--curve", curve, "--setup", setup, "verify", commit, proof, str(int(chunk) + 1), sub, cwd=tmp_path)
    assert r.returncode == 1, r.stderr

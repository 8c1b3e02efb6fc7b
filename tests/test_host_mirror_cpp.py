"""The C++ host mirror (proxmox-backup_amd/host/pbs_chunker.hpp): compiles against the
C ABI on CPU; on the GPU its ChunkStream / DynamicChunkWriter / scan loop / find_cuts
give the oracle's cut list."""
import hashlib
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "host_mirror_main.cpp")
LIBDIR = os.path.join(ROOT, "proxmox-backup_amd", "csrc")


def _build(tmp_path):
    exe = str(tmp_path / "host_mirror")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(ROOT, "proxmox-backup_amd", "host"), SRC, "-L", LIBDIR,
                    "-lpbschunk", f"-Wl,-rpath,{LIBDIR}", "-o", exe], check=True)
    return exe


def test_host_mirror_compiles_and_fails_loudly_without_device(tmp_path, pbschunk):
    exe = _build(tmp_path)
    if pbschunk.device_count() > 0:
        pytest.skip("device visible: covered by the gpu test")
    r = subprocess.run([exe, "65536", "100000", "1", "4096"], capture_output=True, text=True)
    assert r.returncode == 1 and "no HIP device" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("avg,n,piece", [(4096, 3 << 20, 65536), (65536, 9 << 20, 262144), (64, 200000, 1000)])
def test_host_mirror_matches_oracle(tmp_path, gpu, oracle, avg, n, piece):
    exe = _build(tmp_path)
    didx = str(tmp_path / "mirror.didx")
    r = subprocess.run([exe, str(avg), str(n), "7", str(piece)], capture_output=True, text=True, check=True,
                       env={**os.environ, "HOST_MIRROR_DIDX": didx})
    lines = {ln.split(" ", 1)[0]: ln.split()[1:] for ln in r.stdout.strip().splitlines()}
    data = oracle.gen_random(n, 7)
    ref = oracle.chunk_feed(avg, data).tolist()
    assert [int(x) for x in lines["scan"]] == ref
    for tag in ("stream", "stream0", "writer", "batch"):
        ends = [int(x) for x in lines[tag]]
        assert ends[:-1] == ref and ends[-1] == n, tag
    assert "not a power of two" in " ".join(lines["badavg"])
    # DynamicIndexWriter over the writer's chunks == the oracle's .didx restatement
    wends = np.array([int(x) for x in lines["writer"]], dtype=np.uint64)
    bounds = np.concatenate([[0], wends]).astype(np.uint64)
    ref_img, ref_csum = oracle.didx_image(wends, oracle.chunk_digests(data, bounds), bytes(16), 1234)
    assert lines["index"][0] == ref_csum.hex()
    # host CRC-32 of the writer's chunks and the first uncompressed blob's header
    assert [int(x) for x in lines["crc"]] == oracle.chunk_crcs(data, bounds).tolist()
    first = data[:int(wends[0])].tobytes()
    assert lines["blob0"][0] == oracle.blob_uncompressed(first)[:16].hex()
    assert open(didx, "rb").read() == ref_img
    # pipeline_host (copy -> chunk -> digest + CRC) and digest_chunks_host over the buffer
    pends = [int(x) for x in lines["pipe"]]
    assert pends[:-1] == ref and pends[-1] == n
    pb = np.concatenate([[0], np.array(pends, dtype=np.uint64)]).astype(np.uint64)
    want = hashlib.sha256(oracle.chunk_digests(data, pb).tobytes()).hexdigest()
    assert lines["pipedig"][0] == want and lines["hostdig"][0] == want
    assert [int(x) for x in lines["pipecrc"]] == oracle.chunk_crcs(data, pb).tolist()

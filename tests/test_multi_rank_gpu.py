"""The N-rank path with device-bound ranks (BASELINE configs[4]) on the one-GPU test box:
`bench.py --gpus 2` spawns two rank processes before anything touches a GPU; LCRC_RANK_DEVICE_MOD=1 (test-only)
binds rank r to device r % device_count, so both ranks drive the box's one MI355X through their own contexts,
streams and device buffers, exactly the code the driver's 8-GPU run executes with rank r on device r. gloo
carries only the barrier, the max-over-ranks time and the per-rank figures (no data-path collective)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# 4,096 blocks: the launcher; 65,536: BASELINE configs[4]'s per-GPU batch (64K x 4 KiB, 4 rotated 256 MiB buffers per
# rank) -- the size the driver's N-GPU run allocates and streams in every rank -- with rank 0's CPU baseline after the
# timed region, cross-checked against its device CRCs
@pytest.mark.parametrize("NBLK", [4096, 65536])
def test_bench_two_device_ranks(orc, synth, NBLK):
    world = 2
    env = dict(os.environ, LCRC_RANK_DEVICE_MOD="1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--blocks", str(NBLK),
           "--steps", "5" if NBLK == 65536 else "3", "--warmup", "2" if NBLK == 65536 else "1", "--cpu-seconds", "0.5"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    rows = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(rows) == 1, r.stdout  # ONE line, from rank 0 only
    res = json.loads(rows[0])
    print(json.dumps({k: res[k] for k in ("value", "n_gpus", "ms_per_step", "per_gpu", "cpu_baseline")}))
    assert res["n_gpus"] == world and res["scaling"] == "weak"
    assert [g["rank"] for g in res["per_gpu"]] == list(range(world))
    assert [g["device"] for g in res["per_gpu"]] == [0] * world  # rank r on device r % 1
    # each rank's PCI bus ID: the same GPU for both (allowed only under LCRC_RANK_DEVICE_MOD=1)
    bus = [g["pci_bus_id"] for g in res["per_gpu"]]
    assert bus[0] and len(bus[0]) == 12 and bus == [bus[0]] * world
    assert res["roofline"] is not None and res["roofline"]["frac"] > 0
    for g in res["per_gpu"]:
        # each rank checksummed its own batch on the device: its fingerprint is the oracle's (masked CRC-32C)
        data = synth.splitmix_bytes(synth.SEED_FIXED + g["rank"] * 4, NBLK * 4096)
        want = orc.mask_array(orc.crc_ranges(data, np.arange(NBLK, dtype=np.uint64) * 4096, np.full(NBLK, 4096), 1))
        assert g["crc_xor"] == f"{int(np.bitwise_xor.reduce(want)):08x}"
        assert g["launch_us"] > 0 and 0 < g["frac"] < 1.2  # each rank's own launch-carried HIP events
    assert len({g["crc_xor"] for g in res["per_gpu"]}) == world
    cb = res["cpu_baseline"]
    assert cb is not None and cb["matches_device"] is True and cb["cores"] >= 1 and cb["value"] > 0
    assert cb["kind"] == "port" and "cpu_model" in cb
    # the aggregate is all ranks' bytes over the slowest rank's time
    assert abs(res["value"] - world * NBLK * 4096 / (res["ms_per_step"] / 1e3) / 2 ** 30) <= 0.01 * res["value"] + 0.02

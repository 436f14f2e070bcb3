"""N>1 path on the CPU: bench.py end to end with 2 and 4 gloo ranks -- the self-spawning launcher
(`bench.py --gpus N`) and torch.distributed.run -- each rank checksumming its own shard (the path shards with no
data-path collective) through the library's host scalar path (`--engine host`: no device here)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NBLK = 128


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _line(stdout):
    rows = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(rows) == 1, stdout  # ONE line, from rank 0 only
    return json.loads(rows[0])


def _check(orc, synth, res, world, steps):
    assert res["n_gpus"] == world
    assert res["scaling"] == "weak"
    assert [r["rank"] for r in res["per_gpu"]] == list(range(world))
    assert [r["device"] for r in res["per_gpu"]] == list(range(world))  # rank r binds device LOCAL_RANK = r
    # the aggregate is all ranks' bytes over the slowest rank's time
    slowest = min(r["gib_s"] for r in res["per_gpu"])
    assert abs(res["value"] - world * NBLK * 4096 * steps / (res["ms_per_step"] * steps / 1e3) / 2 ** 30) <= \
        0.01 * res["value"] + 0.02
    assert res["value"] >= world * slowest * 0.95
    # each rank checksummed its own shard (independent seeds, no exchange): its fingerprint is the oracle's
    for r in res["per_gpu"]:
        data = synth.splitmix_bytes(synth.SEED_FIXED + r["rank"] * 4, NBLK * 4096)
        want = orc.mask_array(orc.crc_ranges(data, np.arange(NBLK) * 4096, np.full(NBLK, 4096), 1))
        assert r["crc_xor"] == f"{int(np.bitwise_xor.reduce(want)):08x}"
    assert len({r["crc_xor"] for r in res["per_gpu"]}) == world


def _env():
    return dict(os.environ, OMP_NUM_THREADS="1")


@pytest.mark.parametrize("world", [2, 4])
def test_bench_spawns_ranks(orc, synth, world):
    """`python bench.py --gpus N` (no launcher): the script starts the N rank processes itself."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--engine", "host",
           "--blocks", str(NBLK), "--steps", "3", "--warmup", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    _check(orc, synth, _line(r.stdout), world, 3)


@pytest.mark.parametrize("world", [2, 8])
def test_bench_under_torchrun(orc, synth, world):
    """The driver's form: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N -- with N = 8 the
    driver's SCALE run (configs[4]: 8 independent shards, no collective) rehearsed on gloo ranks."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--engine", "host", "--blocks", str(NBLK), "--steps", "2", "--warmup", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    _check(orc, synth, _line(r.stdout), world, 2)


def test_queue_grouping():
    """The queued submission: steps split into submissions, at most 32 batches per launch, balanced."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.groups(5, 50, 0) == [(5, 50)]
    assert bench.groups(0, 10, 4) == [(0, 4), (4, 4), (8, 2)]
    assert [len(p) for p in bench.balanced_jobs(list(range(50)))] == [25, 25]
    assert [len(p) for p in bench.balanced_jobs(list(range(32)))] == [32]
    assert [len(p) for p in bench.balanced_jobs(list(range(65)))] == [22, 22, 21]
    assert bench.launches_of(50) == 2 and bench.launches_of(32) == 1


def test_bench_refuses_ranks_on_one_gpu():
    """Two ranks whose devices resolve to one PCI bus ID: bench.py refuses to print a 2-GPU line,
    unless the test-only LCRC_RANK_DEVICE_MOD=1 put them there on purpose; each rank's bus ID is in per_gpu."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--engine", "host", "--blocks", str(NBLK),
           "--steps", "2", "--warmup", "1", "--assume-bus-id", "0000:75:00.0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=_env(), cwd=ROOT)
    assert r.returncode != 0 and "ranks share a GPU" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=dict(_env(), LCRC_RANK_DEVICE_MOD="1"),
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    res = _line(r.stdout)
    assert [g["pci_bus_id"] for g in res["per_gpu"]] == ["0000:75:00.0"] * 2


def test_bus_id_codes():
    sys.path.insert(0, ROOT)
    import bench
    for s in ("0000:75:00.0", "0001:e5:1f.7", "ffff:00:00.1"):
        assert bench.bus_id_text(float(bench.bus_id_code(s))) == s
    bench.check_distinct_devices([bench.bus_id_code("0000:05:00.0"), bench.bus_id_code("0000:15:00.0"), -1, -1],
                                 False)
    with pytest.raises(SystemExit):
        bench.check_distinct_devices([bench.bus_id_code("0000:05:00.0")] * 2, False)
    bench.check_distinct_devices([bench.bus_id_code("0000:05:00.0")] * 2, True)

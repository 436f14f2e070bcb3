"""N>1 path on the CPU: 2 and 4 gloo ranks through bench.py's barrier / max-over-ranks / aggregate logic, each on
an independent shard (the path shards with no data-path collective)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 4])
def test_multi_rank_gloo(orc, synth, tmp_path, world):
    env = dict(os.environ, OMP_NUM_THREADS="1", LCRC_DIST_OUT=str(tmp_path))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "tests", "_dist_worker.py")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    rows = [json.load(open(tmp_path / f"rank{i}.json")) for i in range(world)]
    assert sorted(x["rank"] for x in rows) == list(range(world))
    # every rank sees the same max-over-ranks time, so the same aggregate value
    assert len({x["elapsed_max"] for x in rows}) == 1
    assert abs(rows[0]["value"] - world * 256 * 4096 * 3 / rows[0]["elapsed_max"] / 2 ** 30) < 1e-6
    # each rank checksummed its own shard (weak scaling: independent seeds, no exchange)
    for x in rows:
        data = synth.splitmix_bytes(synth.SEED_FIXED + x["rank"], 256 * 4096)
        want = orc.crc_ranges(data, np.arange(256) * 4096, np.full(256, 4096), 1)
        assert x["xor"] == int(np.bitwise_xor.reduce(want))
    assert len({x["xor"] for x in rows}) == world

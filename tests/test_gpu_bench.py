"""The benchmark checks the kernel it times (pytest -m gpu).

bench.py's headline step is two k_step launches, one per HIP stream, each sealing and then
opening half of C1 (65,536 x 1,420 B, one key). Each half is 32,768 packets, so its grid is
half the resident waves and the launch takes the k_step<8, 4> build (wg_capi.hip,
launch_after_seal). These tests pin that exact shape against the oracle, and show that the
bench line's own check (`verified`, `oracle_sample`) fails when k_step writes a wrong tag
(test hook WG_TEST_STEP_FLIP).

Reference: ChaCha20Poly1305.java:31-60 (poly1305AeadEncrypt / Decrypt), SymmetricKeypair.java:52-83
(nonce = LE64(counter) || 0^4).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from wgtest import ROOT, oracle, splitmix_np, wg

pytestmark = pytest.mark.gpu
O = oracle()


def test_bench_two_stream_step_every_packet_vs_oracle(engine):
    """The bench's timed shape: two streams, each one WG_F_AFTER_SEAL k_step over 32,768 packets of
    shared buffers; three steps in a row so launches of different steps overlap. Every ct || tag is
    compared with the oracle, every plaintext with the input, every status must be OK."""
    import torch
    W = wg()
    dev = torch.device("cuda", 0)
    n, L, stride = 65536, 1420, 1440
    keys = splitmix_np(0xC0FFEE, 32)
    engine.set_keys(0, keys.tobytes())
    off = np.arange(n, dtype=np.uint64) * stride
    desc = W.pack_desc(off, off, np.arange(n, dtype=np.uint64), L, 0)
    pt = splitmix_np(0x5EED, n * stride)
    d_desc = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
    d_pt = torch.from_numpy(pt).to(dev)
    d_ct = torch.full((n * stride,), 0x5A, dtype=torch.uint8, device=dev)
    d_back = torch.full((n * stride,), 0xA5, dtype=torch.uint8, device=dev)
    status = torch.full((n,), -1, dtype=torch.int32, device=dev)
    main = torch.cuda.current_stream()
    side = [torch.cuda.Stream(device=dev) for _ in range(2)]
    cuts = [0, n // 2, n]
    for s_ in side:
        s_.wait_stream(main)
    for _ in range(3):
        for i, s_ in enumerate(side):
            a, b = cuts[i], cuts[i + 1]
            with torch.cuda.stream(s_):
                engine.duplex(d_desc[a:b], d_pt, d_ct, L, d_desc[a:b], d_ct, d_back, status[a:b], L,
                              uniform=True, after_seal=True)
    for s_ in side:
        main.wait_stream(s_)
    torch.cuda.synchronize()
    ref = np.zeros(n * stride, np.uint8)
    O.seal_batch(desc, pt, ref, keys, threads=16)
    ct = d_ct.cpu().numpy().reshape(n, stride)
    ref = ref.reshape(n, stride)
    bad = np.nonzero(~np.all(ct[:, :L + 16] == ref[:, :L + 16], axis=1))[0]
    assert bad.size == 0, f"{bad.size} packets' ct||tag differ from the oracle (first {bad[:8]})"
    assert not status.cpu().numpy().any()
    back = d_back.cpu().numpy().reshape(n, stride)
    assert np.array_equal(back[:, :L], pt.reshape(n, stride)[:, :L])


def _bench(extra_env, steps="2", *extra):
    env = dict(os.environ, **extra_env)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", steps, "--warmup", "1",
                        "--ramp-ms", "0", *extra], cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert lines, f"no JSON line (rc {p.returncode}): {p.stderr[-2000:]}"
    return p.returncode, json.loads(lines[-1])


def test_bench_line_fails_when_k_step_writes_a_wrong_tag():
    """WG_TEST_STEP_FLIP=64: k_step flips one tag bit of every 64th packet between its seal and open
    halves. The bench line must then report verified false and oracle_sample.bit_exact false, and the
    bench must exit 3. Without the hook the same short run is verified and bit-exact."""
    # the hook exists only in the test library (make -C wireguard-java_amd/csrc test); the product
    # library ignores the variable, which the last run below also shows
    test_lib = os.path.join(ROOT, "wireguard-java_amd", "libwgaead_test.so")
    assert os.path.exists(test_lib), "build the test library first (__graft_entry__.build())"
    rc, line = _bench({"WG_TEST_STEP_FLIP": "64", "WG_LIB_PATH": test_lib})
    assert rc == 3, line
    assert line["verified"] is False
    assert line["oracle_sample"]["bit_exact"] is False
    rc, line = _bench({})
    assert rc == 0, line
    assert line["verified"] is True and line["oracle_sample"]["bit_exact"] is True
    assert line["config"]["streams"] == 2 and line["roofline"]["kernel_names"] == ["k_step"]
    assert line["stagger"] is False and line["window_launches"] == 4 and line["spin_sync"] is True
    # the staggered two-stream schedule (--stagger 1): 2 steps = 2 launches on stream A, Q1 + 1 window + Q2 on B
    for steps in ("1", "2", "3"):
        rc, line = _bench({}, steps, "--stagger", "1")
        assert rc == 0 and line["verified"] is True and line["oracle_sample"]["bit_exact"] is True, line
        assert line["stagger"] is True and line["window_launches"] == 2 * int(steps) + 1
    rc, line = _bench({"WG_TEST_STEP_FLIP": "64"})  # the product library: no hook, still bit-exact
    assert rc == 0 and line["verified"] is True and line["oracle_sample"]["bit_exact"] is True


def test_bench_imix_fused_planning_is_verified():
    """WG_LPT_FUSED=1 (A/B knob, off by default): the IMIX step's short-packet plan made by the step launch's
    own first workgroups (k_step_mixed_fused) while the others wait on its publication count, with each poll
    kind (WG_FUSED_POLL 0/1/2) and planner count (WG_FUSED_NP): every packet must still round-trip and the
    oracle sample be bit-exact, as on the default two-launch plan."""
    for env in ({}, {"WG_LPT_FUSED": "1"}, {"WG_LPT_FUSED": "1", "WG_FUSED_POLL": "2", "WG_FUSED_NP": "256"},
                {"WG_LPT_FUSED": "1", "WG_FUSED_POLL": "1", "WG_FUSED_NP": "7"}):
        rc, line = _bench(env, "3", "--workload", "imix")
        assert rc == 0 and line["verified"] is True and line["oracle_sample"]["bit_exact"] is True, (env, line)


def test_bench_imix_two_streams_own_workspaces():
    """IMIX on two streams (--streams 2): each stream's k_lpt_one plans into its own workspace (WG_STREAM_WS,
    on by default), so the halves run concurrently; with WG_STREAM_WS=0 they share one workspace and wait for
    each other. Every packet of both halves must round-trip and the oracle sample be bit-exact either way."""
    for env in ({}, {"WG_STREAM_WS": "0"}):
        rc, line = _bench(env, "3", "--workload", "imix", "--streams", "2")
        assert rc == 0 and line["verified"] is True and line["oracle_sample"]["bit_exact"] is True, (env, line)
        assert line["config"]["streams"] == 2


def test_bench_imix_graph_is_verified():
    """IMIX captured into a HIP graph (--graph): the capture stream has no plan workspace of its own and cannot
    allocate one, so it plans in the shared workspace the earlier calls sized; every packet must round-trip."""
    rc, line = _bench({}, "3", "--workload", "imix", "--graph")
    assert rc == 0 and line["verified"] is True and line["oracle_sample"]["bit_exact"] is True, line
    assert line["graph"] is True

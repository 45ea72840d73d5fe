"""Host sanitizers over the oracle: oracle/ggrs_oracle.c built with -fsanitize=address,undefined
(GPU sanitizers are not available on this pool; the C restatement is the host code that matters),
driven by oracle/sanitize_main.c; its digests must equal the normal build's."""
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def test_oracle_under_asan_ubsan(oracle, tmp_path):
    exe = str(tmp_path / "oracle_asan")
    subprocess.run(["gcc", "-O1", "-g", "-ffp-contract=off", "-fno-omit-frame-pointer", "-std=c11", "-D_GNU_SOURCE",
                    "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                    os.path.join(ROOT, "oracle", "ggrs_oracle.c"), os.path.join(ROOT, "oracle", "sanitize_main.c"),
                    "-o", exe, "-lm", "-lpthread"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert r.returncode == 0, r.stderr
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
    lines = dict((" ".join(l.split()[:2]) if l.startswith("synctest") else l.split()[0], l) for l in r.stdout.splitlines())
    # same digests from the normal (ctypes) build
    cases = [(2, 8, 7, 2, 400, 0), (4, 9, 8, 0, 300, 1), (1, 4, 2, 1, 200, 0), (3, 63, 62, 0, 150, 1)]
    for c, (P, mp, cd, d, frames, model) in enumerate(cases):
        inp = oracle.gen_inputs(0x6767525300000000 + c, frames, P, model)
        res = oracle.synctest_run(inp, P, mp, cd, d, corrupt_frame=77 if c == 1 else -1)
        done = res["result"].frames_done
        want = (f"synctest {c} status {res['result'].status} frames {done} last "
                f"{int(res['cksum'][done - 1])} final {oracle.fletcher16(bytes(res['final_state']))}")
        assert lines[f"synctest {c}"] == want
    pr = oracle.particles_synctest_run(oracle.gen_inputs(9, 40, 2, 1), 64, 2, 17, 16, session=3)
    assert lines["particles"] == (f"particles status {pr['result'].status} last {int(pr['ck_trace'][39])} "
                                  f"final {oracle.fletcher16(bytes(pr['final_state']))}")
    _, cks, _ = oracle.p2p_replay(oracle.state_new(2), 0, np.array([(i * 5) % 16 for i in range(16)], np.uint8))
    assert lines["p2p"] == f"p2p last {int(cks[7])}"

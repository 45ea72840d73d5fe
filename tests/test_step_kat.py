"""CPU KAT of the arithmetic identity the v4 SyncTest step relies on: the speed clamp test
`sqrtf(vx*vx + vy*vy) > 7` (ex_game.rs:313-317) equals `vx*vx + vy*vy > 49` for every f32
(2^32 inputs, a few seconds on 8 cores), so the square root is only taken inside the clamp."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_clamp_test_equivalence_every_f32(tmp_path):
    exe = str(tmp_path / "step_kat_host")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-o", exe,
                    os.path.join(HERE, "native", "step_kat_host.c"), "-lm", "-lpthread"], check=True)
    r = subprocess.run([exe, str(min(8, os.cpu_count() or 1))], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip() == "bad 0"


def test_turn_rem_euclid_every_rotation_in_domain(tmp_path):
    """The lean step's turn `a < 0 ? a + 2pi : (a >= 2pi ? a - 2pi : a)` equals
    f32::rem_euclid(rot -/+ ROTATION_SPEED, 2pi) (ex_game.rs:300-306) for every f32 rot in
    [+0, 2pi], both directions."""
    exe = str(tmp_path / "remeuclid_kat_host")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-o", exe,
                    os.path.join(HERE, "native", "remeuclid_kat_host.c"), "-lm", "-lpthread"], check=True)
    r = subprocess.run([exe, str(min(8, os.cpu_count() or 1))], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip() == "bad 0"

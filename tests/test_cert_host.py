"""Host-side checks of the certification self-test inputs (tests/cert_cases.py) and of the phase-C bound itself.

* oracle_auxa_boundary returns the reference's exact CDF boundary: the pick at it exceeds the entry, the pick one
  double below does not (mcmc.c:901-915's sequential subtractions);
* phase C's decision rule (pc_classify / pc_resolve, restated on the host in cert_cases.emulate_decide) never
  decides against the reference on the threshold-crossing proposals, and with its margin divided by 2^8 it does --
  the generated cases reach the band an understated bound fails in (the GPU test runs the device code itself)."""
import numpy as np

import cert_cases
import oracle_ref


def test_boundary_is_the_reference_boundary():
    rng = np.random.default_rng(5)
    for N, kind in ((256, "random"), (256, "tail"), (600, "steep"), (1500, "random")):
        col, rev, o, L = cert_cases.gibbs_block_columns(kind, N, rng)
        x = cert_cases.walk_bits(col, N, rev, L)
        for c, d in cert_cases.cd_grid()[::5]:
            _, p = oracle_ref.auxa_pick(x, o, c, d, 0.5, want_p=True)
            for i in sorted(set([int(np.argmax(p)), 0, L - 1, o])):
                if not 0 <= i < L:
                    continue
                ub = oracle_ref.auxa_boundary(x, o, c, d, i)
                if ub > 1.0:
                    continue
                assert oracle_ref.auxa_pick(x, o, c, d, ub) > i
                if ub > 0.0:
                    assert oracle_ref.auxa_pick(x, o, c, d, float(np.nextafter(ub, 0.0))) <= i


def test_phase_c_bound_holds_and_a_shrunken_one_fails():
    cs = cert_cases.decide_cases(3, n_combos=24)
    assert cs["n"] >= 300
    got = cert_cases.emulate_decide(cs)
    decided = got != 3
    assert decided.sum() >= cs["n"] // 4
    assert (got[decided] == cs["expected"][decided]).all()
    shrunk = cert_cases.emulate_decide(cs, shift=8)
    d8 = shrunk != 3
    assert (shrunk[d8] != cs["expected"][d8]).any(), "the cases never reach the band an Eb / 2^8 bound fails in"

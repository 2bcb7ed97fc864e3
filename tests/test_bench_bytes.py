"""bench.py's byte models (no GPU): SURVEY.md §8(d)'s per-agent-step figure
B_as, which prices a launch that runs whole steps, at the BASELINE shapes; and
the rollout's own per-step count, which must stay below it (its state stays on
chip)."""
import pytest

import bench


@pytest.mark.parametrize("N,No,edges_per_env,expect", [(24, 24, 92.59, 191.3), (96, 96, 387.91, 193.5),
                                                       (3, 3, 10.7, 187.8)])
def test_survey_bytes_per_agent_step(N, No, edges_per_env, expect):
    B = 1024
    b_as = bench.survey_bytes_per_agent_step(N, No, 4, edges_per_env * B, B)
    # 32 + A + 8 + 8 No/N + 9 + (E/N) F 4 + 12 e, e = edges per agent
    E = 2 * N + No
    assert b_as == pytest.approx(32 + 4 + 8 + 8 * No / N + 9 + E / N * 28 + 12 * edges_per_env / N)
    assert b_as == pytest.approx(expect, abs=0.1)


@pytest.mark.parametrize("N,No,seg", [(24, 24, True), (96, 96, False), (3, 3, True)])
def test_rollout_moves_fewer_bytes_than_a_step(N, No, seg):
    B, edges = 8192, 4.0 * N * 8192
    roll = bench.roll_step_bytes(B, N, No, 100, 4, edges, seg)
    full = bench.survey_bytes_per_agent_step(N, No, 4, edges, B) * B * N
    assert 0 < roll < full

"""Host-side duration of each TrainingSession.step() call at C2 (does the host run ahead of the GPU
or block in a call?).  python tools/host_step_timing.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from spectralmc_amd.gbm_trainer import GbmCVNNPricer  # noqa: E402
from spectralmc_amd.models.numerical import Precision  # noqa: E402
from tests.helpers import (expect_success, make_black_scholes_config, make_domain_bounds,  # noqa: E402
                           make_gbm_cvnn_config, make_simulation_params, make_test_cvnn, make_training_config)


def main() -> None:
    lanes = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    B, T, N, M = 4096, 16, 256, 256
    sp = make_simulation_params(timesteps=T, network_size=N, batches_per_mc_run=M, threads_per_block=256, mc_seed=7,
                                buffer_size=512, dtype=Precision.float32)
    model = make_test_cvnn(n_inputs=6, n_outputs=N, seed=123, dtype=torch.float32, device="cuda:0", hidden_layers=2,
                           hidden_width=32)
    cfg = make_gbm_cvnn_config(model, sim_params=sp, bs_config=make_black_scholes_config(sim_params=sp),
                               domain_bounds=make_domain_bounds())
    pricer = expect_success(GbmCVNNPricer.create(cfg))
    pricer.mc_lanes = lanes
    pricer.math_mode = "hw"
    session = expect_success(pricer.open_session(make_training_config(num_batches=40, batch_size=B, learning_rate=1e-2)))
    for _ in range(4):
        expect_success(session.step())
    session.sync()
    torch.cuda.synchronize()
    ts = []
    t0 = time.perf_counter()
    for _ in range(20):
        a = time.perf_counter()
        expect_success(session.step())
        ts.append((time.perf_counter() - a) * 1e3)
    t_enq = (time.perf_counter() - t0) * 1e3
    session.sync()
    torch.cuda.synchronize()
    t_all = (time.perf_counter() - t0) * 1e3
    print("host ms per step() call:", " ".join(f"{x:.2f}" for x in ts))
    print(f"lanes={lanes}: enqueue of 20 steps {t_enq:.1f} ms, until done {t_all:.1f} ms ({t_all / 20:.3f} ms/step)")
    session.close()


if __name__ == "__main__":
    main()

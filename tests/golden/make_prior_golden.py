"""G8 (g8_prior_draws.npz): draws of the reference's own prior sampler, for the synthetic-TAC generator (f3).

Run in the build container only (needs /root/reference, read-only):
    python tests/golden/make_prior_golden.py

* ``dvr_raw`` / ``r1_raw``: helper_func.truncnormal_samples (helper_func.py:153-162) on the reference's
  prior (G0: mu_DVR / Cov_DVR, mu_R1 / Cov_R1 of prior_stats_nROI48.pik), cond_test None as for the
  training set (sample_sim_data.py:136-137), seeded through the global np.random state it draws from.
* ``dvr_sel`` / ``r1_sel``: the selection sample_sim_data.py:139-188 applies on top: DVR, R1 and the
  reference TAC drawn by truncnormal_samples, then, per sample, the three redrawn (again by
  truncnormal_samples) while kinetic_model.SRTM2.create_activity_curve * dt (kinetic_model.py:142-158)
  has a negative frame.  The loop below calls the reference's functions in the reference's order; the
  saved arrays are their outputs.

helper_func imports NP_DTYPE from diffusion_model (TensorFlow, absent here), so the same stub module as
make_golden.py's G1 is inserted first.  Only draws are stored (data, no reference source).
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = '/root/reference'
N_RAW, N_SEL = 2000, 2000
SEED_RAW, SEED_SEL = 20261018, 20261019


def main():
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from pet_posterior_distribution_amd.sim_data import reference_prior, time_grid
    stub = types.ModuleType('diffusion_model')
    stub.NP_DTYPE = np.float32
    sys.modules['diffusion_model'] = stub
    sys.path.insert(0, REF)
    import helper_func as hf
    import kinetic_model as km

    pr = reference_prior()
    tv, dt = time_grid()
    inv = np.linalg.inv
    np.random.seed(SEED_RAW)
    dvr_raw = np.asarray(hf.truncnormal_samples(pr['mu_DVR'], pr['Cov_DVR'], inv(pr['Cov_DVR']), N_RAW))
    r1_raw = np.asarray(hf.truncnormal_samples(pr['mu_R1'], pr['Cov_R1'], inv(pr['Cov_R1']), N_RAW))

    # sample_sim_data.py:139-188 with cond_test None (training data)
    np.random.seed(SEED_SEL)
    args = lambda k: (pr['mu_' + k], pr['Cov_' + k], inv(pr['Cov_' + k]))   # noqa: E731
    varDVR = hf.truncnormal_samples(*args('DVR'), N_SEL)
    varR1 = hf.truncnormal_samples(*args('R1'), N_SEL)
    vartacref = hf.truncnormal_samples(*args('tac_ref'), N_SEL)
    redraws = 0
    for i in range(N_SEL):
        while True:
            model = km.SRTM2(frame_time_list=tv, frame_duration_list=dt, tac_reference=vartacref[i])
            x = (model.create_activity_curve(DVR=varDVR[i], R1=varR1[i], k2p=pr['mu_k2p']) * dt[:, None]).T
            if not (x < 0).any():
                break
            redraws += 1
            varDVR[i] = hf.truncnormal_samples(*args('DVR'), 1)[0]
            varR1[i] = hf.truncnormal_samples(*args('R1'), 1)[0]
            vartacref[i] = hf.truncnormal_samples(*args('tac_ref'), 1)[0]
    np.savez(os.path.join(HERE, 'g8_prior_draws.npz'), dvr_raw=dvr_raw, r1_raw=r1_raw,
             dvr_sel=np.asarray(varDVR), r1_sel=np.asarray(varR1), redraws=np.int64(redraws),
             seeds=np.array([SEED_RAW, SEED_SEL], dtype=np.int64))
    print('g8:', dvr_raw.shape, r1_raw.shape, len(varDVR), 'redraws', redraws)


if __name__ == '__main__':
    main()

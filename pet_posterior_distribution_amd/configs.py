"""Configuration of record of the reference (main_script.py:131-186)."""


def shipped_net_args():
    """net_args of main_script.py:135-167 (iDDPM f128/d4, learn_ranged)."""
    return {
        'num_channels_out': 2, 'learn_variance': 'learn_ranged', 'num_filt_start': 128, 'pool_size': 2,
        'depth': 4, 'block_type': 'conv', 'block_params': {'flag_res': True, 'kernel_size': 6},
        'cond_params': {'flag_flatten_input': False, 'network_name': 'encoder',
                        'network_kwargs': {'enc_size': [256, 128, 64], 'latent_dim': 32,
                                           'final_activation': None}},
        'skip_conn_type': 'concat', 'skip_conn_op': None, 'skip_conn_post_op': None, 'dropout': None,
        'final_activation': None, 'sin_emb_dim': 64, 'normalize_feature_dict': None,
        'normalize_label_dict': None}


def shipped_diff_args():
    """diff_args of main_script.py:179-186."""
    return {'timesteps': 1000, 'noise_schedule': {'schedule_name': 'cosine'}, 'lambda_vlb': 1e-1, 'ndim': 1}

"""Default configurations (reference red_diffeq/config/default_config.py:3-69)."""
from .config_dict import ConfigDict


def get_config():
    c = ConfigDict()
    c.pde = ConfigDict(n_grid=70, nt=1000, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=70, ns=5)
    c.model = ConfigDict(dim=64, dim_mults=(1, 2, 4, 8), flash_attn=False, channels=1)
    c.diffusion = ConfigDict(image_size=72, timesteps=1000, sampling_timesteps=250, objective="pred_noise",
                             model_path="pretrained_models/model-4.pt")
    c.optimization = ConfigDict(lr=0.03, ts=300, diffusion_ts=1, regularization="diffusion", reg_lambda=0.75,
                                use_time_weight=False, fixed_timestep=None, sigma=10.0, sigma_x0=0.0001,
                                initial_type="smoothed", noise_std=0.0, noise_type="gaussian", missing_number=0)
    c.data = ConfigDict(seismic_data_dir="dataset/OpenFWI/Seismic_Data/",
                        velocity_data_dir="dataset/OpenFWI/Velocity_Data/", batch_size=1, data_pattern="*.npy",
                        use_mmap=True)
    c.experiment = ConfigDict(name="red_diffeq_default", results_dir="experiment/", save_intermediate=False,
                              log_interval=10, save_metrics=True, random_seed=None)
    return c


def get_marmousi_config():
    c = get_config()
    c.data.seismic_data_dir = "dataset/Marmousi/Seismic_Data/"
    c.data.velocity_data_dir = "dataset/Marmousi/Velocity_Data/"
    c.data.batch_size = 1
    c.experiment.name = "marmousi_inversion"
    return c

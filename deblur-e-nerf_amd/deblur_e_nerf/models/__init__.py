from . import deblur_e_nerf, event_generation_params, nerf, pixel_bandwidth, trajectories  # noqa: F401

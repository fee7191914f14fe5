"""nicecore — MI355X-native render core for NICE-SLAM's Renderer.render_batch_ray.

Public surface (drop-in for the reference's renderer / decoder APIs):
  nicecore.renderer.Renderer       src/utils/Renderer.py
  nicecore.decoder.NICE / MLP / MLP_no_xyz / get_model
                                   src/conv_onet/models/decoder.py, src/conv_onet/config.py
  nicecore.ops.render_rays / eval_points   functional forms
  nicecore.scene                   bounds, grid shapes/init, presets, synthetic rays
  nicecore.distributed             ray-sharded data parallelism over RCCL
"""
__version__ = "0.1.0"

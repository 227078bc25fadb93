"""svo_amd — MI355X-native direct-alignment hot path of amin-abouee/semi-direct-visual-odometry.

Product path: HIP kernels in libsvo_hip.so behind the C ABI of include/svo_c.h.  This package mirrors the
reference's ImagePyramid / ImageAlignment / FeatureAlignment class surface over that ABI (core.py).
"""
from .core import (DEPTH_SEED, MEDIAN_EXACT, MEDIAN_REFERENCE, SCALE_AUTO, SCALE_K2, SCALE_K2R, SCALE_K2V, SCALE_K2V_LAYA_SLOTS, SCALE_K2V_LAYB_SLOTS, SCALE_K2V_MAX_SLOTS, AlignBatch, BundleAdjustment, Context, DepthEstimator, Feature, FeatureAlignment, FeatureSelection, Frame,
                   ImageAlignment,
                   ImagePyramid, Map, PinholeCamera, Point, PointType, PyramidSet, default_context, depth_seeds,
                   debug_robust_scale, depth_update, device_count, pose_optimize_batch, robust_scale_capacity)
from ._capi import STATUS_NAMES, SvoError

__all__ = ["DEPTH_SEED", "MEDIAN_EXACT", "MEDIAN_REFERENCE", "SCALE_AUTO", "SCALE_K2R", "SCALE_K2V", "SCALE_K2V_MAX_SLOTS", "SCALE_K2V_LAYA_SLOTS", "SCALE_K2V_LAYB_SLOTS", "SCALE_K2", "robust_scale_capacity", "debug_robust_scale", "AlignBatch", "BundleAdjustment", "pose_optimize_batch", "Context", "DepthEstimator", "depth_seeds", "depth_update", "Feature", "FeatureAlignment", "FeatureSelection", "Frame", "ImageAlignment", "ImagePyramid",
           "Map", "PinholeCamera", "Point", "PointType", "PyramidSet", "default_context", "device_count", "STATUS_NAMES", "SvoError"]

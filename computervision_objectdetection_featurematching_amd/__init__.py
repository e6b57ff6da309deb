"""MI355X-native brute-force L2 kNN(k=2) matcher + Lowe ratio test + RANSAC homography.

Drop-in for the hot path of mattreturn1/ComputerVision_ObjectDetection_FeatureMatching
(src/TestsDetector.cpp:36-95).  C ABI: include/mim.h (libmim.so); Python mirror: matcher.py.
"""
from .matcher import DMatch, Matcher, default_params  # noqa: F401

__all__ = ["Matcher", "DMatch", "default_params"]

"""acoss (MI355X engine) — drop-in for the acoss cover-song benchmark's all-pairs hot path.

Mirrors the reference package layout (silvadirceu/acoss-1: acoss.coverid,
acoss.algorithms.*, acoss.utils) so user code keeps its imports; the per-pair work runs as
HIP kernels for gfx950 behind the C-ABI in include/acoss_hip.h (see acoss._lib).

Put the directory that contains this package (acoss-1_amd/) on sys.path.
Unlike the reference's acoss/__init__.py, importing the package does not pull in the
audio feature extractors (essentia/librosa/madmom), which are out of scope here.
"""
__version__ = "0.1.0+mi355x"

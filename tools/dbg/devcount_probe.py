"""Probe: does loading the ablation library or torch's HIP init change libccmm's device count?"""
import ctypes
import sys

sys.path.insert(0, ".")
import __graft_entry__ as g

pkg = g.load_package()
lib = pkg.load_library()
print("libccmm device count", lib.ccmm_device_count())
abl = ctypes.CDLL("ccmmshadowratevar-code_amd/csrc/libccmm_ablation.so")
print("after ablation load", lib.ccmm_device_count(), abl.ccmm_device_count())
import torch
print("torch", torch.cuda.is_available(), lib.ccmm_device_count())

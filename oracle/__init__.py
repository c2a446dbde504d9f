"""TEST INFRASTRUCTURE ONLY -- the CPU oracle for the U-Net hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker / CPU baseline.  The product
path (hcunet_amd/, hcat/) never imports it.
"""

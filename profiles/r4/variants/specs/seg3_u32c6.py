import runpy, os
U32 = runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "seg3_u32.py"))["U32"]
SUBS = U32 + [("""  hipLaunchKernelGGL(k_seg_stream<>, dim3(grid), dim3(kFastThreads), 0, s, b.base, b.off, b.len, n, lg_chunk, plan_bad,""",
"""  hipLaunchKernelGGL(k_seg_stream<>, dim3(grid), dim3(kFastThreads), 0, s, b.base, b.off, b.len, n, lg_chunk - 1, plan_bad,""")]

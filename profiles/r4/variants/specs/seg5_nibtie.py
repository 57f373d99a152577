import runpy, os
d = os.path.dirname(os.path.abspath(__file__))
SUBS = runpy.run_path(os.path.join(d, "seg5_nib.py"))["NIB"] + runpy.run_path(os.path.join(d, "seg5_tie.py"))["TIE"]

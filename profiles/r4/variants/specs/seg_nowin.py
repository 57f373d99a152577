SUBS = [("    if (evm) events(we, rs, wpos, evm);\n", "    (void)evm;\n"),
        ("    wraw = win_issue(nf);\n", "")]

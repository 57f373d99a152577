SUBS = [("    if (evm) events(we, rs, wpos, evm);\n", "    (void)evm;\n")]

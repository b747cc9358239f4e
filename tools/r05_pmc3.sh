#!/bin/bash
# round 5: counters of the final tree kernel (CF, C6) for VALU / LDS per 64 packets
bash tools/pmc_probe.sh CF_tree_final CF:tree sq sq2 clk && bash tools/pmc_probe.sh C6_tree_final C6:tree sq sq2 clk && echo pmc3_done

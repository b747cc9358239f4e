#!/bin/bash
# round 5: counters of the tree kernel vs the list / scan kernels on configs C (flows), C6, C3
bash tools/pmc_probe.sh CF_tree CF:tree && bash tools/pmc_probe.sh C6_tree C6:tree && \
bash tools/pmc_probe.sh C6_scan C6:scan && bash tools/pmc_probe.sh C3_tree C3:tree && \
bash tools/pmc_probe.sh C3_scan C3:scan && echo pmc_done

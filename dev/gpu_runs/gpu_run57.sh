#!/bin/bash
# glds engine grid-size threshold A/B (PDNN_GLDS_MIN_TILES 192/256/320/400/600): 192 best (7744-7751 vs 7675-7695)

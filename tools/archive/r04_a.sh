#!/bin/bash
bash tools/r04_base.sh && bash tools/r04_diag.sh

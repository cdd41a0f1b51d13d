REPS=2 AB_SCENES='bunny 1920 1080 64;sponza 1920 1080 64' bash scripts/ab_run.sh ${1:-ab} 3

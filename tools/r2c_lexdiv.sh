# A/B of the lexicon-loop entry rule (GBPE_LEXICON_DIV) on C5, the headline and C2
export TMPDIR=/tmp
for spec in "d16:GBPE_LEXICON_DIV=16" "d8:GBPE_LEXICON_DIV=8" "d4:GBPE_LEXICON_DIV=4" "d2:GBPE_LEXICON_DIV=2"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs EXPLORE_REPS=1 timeout -k 10 200 python tools/explore_1g.py code1g > gpurun_out/ld_$name.log 2>&1 || exit 1
done
for spec in "d16:GBPE_LEXICON_DIV=16" "d4:GBPE_LEXICON_DIV=4"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs EXPLORE_REPS=1 timeout -k 10 200 python tools/explore_1g.py en1g c2 > gpurun_out/ldh_$name.log 2>&1 || exit 1
done

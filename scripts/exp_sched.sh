echo headline; bash scripts/ab_libs.sh "base ilp trk"
echo c4; bash scripts/ab_libs.sh "base ilp trk" --topology geant --policy dqn_buffer --ping-as-obs 0 --replicas 2048
echo c5; bash scripts/ab_libs.sh "base ilp trk" --topology er256 --policy dqn_buffer --warmup 13

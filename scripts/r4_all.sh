# passes 6-8 in one box acquisition
bash scripts/r4_gpu6.sh && bash scripts/r4_gpu7.sh && bash scripts/r4_gpu8.sh

set -u
mkdir -p gpurun_out/s5
for st in 20 200; do
timeout -k 10 900 tools/ab_env.sh $st "base:MIRT_X=0|adapt:MIRT_ADAPTIVE_GRID=1|sdma:MIRT_D2H=sdma|adapt_sdma:MIRT_ADAPTIVE_GRID=1 MIRT_D2H=sdma|base2:MIRT_X=0|adapt2:MIRT_ADAPTIVE_GRID=1" > gpurun_out/s5/ab_$st.log 2>&1; echo "ab $st rc=$?"
cat gpurun_out/s5/ab_$st.log
done

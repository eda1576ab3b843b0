set -u
export TMPDIR=/tmp
rm -f gpurun_out/cb_mf.txt
for s in head layer1 layer2 layer3 layer4; do
timeout -k 10 200 ./tools/convbench 20 "$s" >> gpurun_out/cb_mf.txt 2>&1 || { echo convbench failed; exit 1; }
done
cat gpurun_out/cb_mf.txt

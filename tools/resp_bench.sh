#!/bin/bash
# End-to-end RESP throughput (GPU box, repo root): start sk-resp-server, drive it with tools/resp_load.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/resp
mkdir -p $O
timeout -k 5 300 ./redisson_amd/sk-resp-server --port 0 > $O/server.out 2> $O/server.err &
SP=$!
for i in $(seq 1 100); do grep -q ready $O/server.out 2>/dev/null && break; sleep 0.2; done
PORT=$(sed -n 's/^ready .*:\([0-9]*\)$/\1/p' $O/server.out)
[ -n "$PORT" ] || { echo "server did not start"; cat $O/server.err; kill $SP; exit 1; }
rc=0
for args in "--op pfadd --conns 1 --cmds 1048576" "--op pfadd --conns 4 --cmds 1048576" "--op getbit --conns 4 --cmds 1048576"; do
  timeout -k 5 120 ./tools/resp_load --port $PORT $args >> $O/load.jsonl || { rc=1; break; }
done
kill $SP; wait $SP
cat $O/load.jsonl
exit $rc

/*
 * GpuSketchBatchService -- RBatch executor for sketch commands.
 *
 * CommandBatchService queues (BatchCommandData) per slot with a global index
 * (M:command/CommandBatchService.java:91-111) and answers in enqueue order
 * (:163-171).  This subclass executes the sketch commands of the batch on the
 * GPU instead: the queue is replayed in index order, consecutive commands of
 * the same kind (PFADD / GETBIT / SETBIT / PFCOUNT) become ONE device batch
 * (exact sequential replies inside the batch, sk_pfadd / sk_setbit), and any
 * error fails the whole batch future with the last error, as CommandDecoder
 * does (M:client/handler/CommandDecoder.java:183-197).  Non-sketch commands of
 * the same batch still go to redis-server through super.executeAsync().
 * Source only here; see INTEGRATION.md.
 */
package org.redisson.gpu;

import java.util.ArrayList;
import java.util.HashSet;
import java.util.List;
import java.util.Set;

import org.redisson.client.RedisException;
import org.redisson.client.codec.Codec;
import org.redisson.client.protocol.RedisCommand;
import org.redisson.command.CommandBatchService;
import org.redisson.connection.ConnectionManager;
import org.redisson.connection.NodeSource;

import io.netty.util.concurrent.Future;
import io.netty.util.concurrent.Promise;

public class GpuSketchBatchService extends CommandBatchService {

    static final class Cmd {
        final Codec codec;
        final RedisCommand<?> command;
        final Object[] params;
        final Promise<Object> promise;

        @SuppressWarnings("unchecked")
        Cmd(Codec codec, RedisCommand<?> command, Object[] params, Promise<?> promise) {
            this.codec = codec;
            this.command = command;
            this.params = params;
            this.promise = (Promise<Object>) promise;
        }
    }

    final long ctx;
    final List<Cmd> sketch = new ArrayList<Cmd>();
    final Set<String> touched = new HashSet<String>();

    public GpuSketchBatchService(ConnectionManager connectionManager, long ctx) {
        super(connectionManager);
        this.ctx = ctx;
    }

    @Override
    protected <V, R> void async(boolean readOnlyMode, NodeSource nodeSource, Codec codec, RedisCommand<V> command,
                                Object[] params, Promise<R> mainPromise, int attempt) {
        String name = command.getName();
        // GET / SET / DEL join the sketch queue when the engine holds the key, or an earlier sketch command of
        // this batch names it (it may create the key before this one runs)
        boolean keyCommand = GpuSketchCommandService.KEY_COMMANDS.contains(name) && params.length > 0
                && (touched.contains(params[0].toString()) || SketchDispatch.engineHolds(ctx, params[0]));
        if (!keyCommand && !GpuSketchCommandService.SKETCH_COMMANDS.contains(name)) {
            super.async(readOnlyMode, nodeSource, codec, command, params, mainPromise, attempt);
            return;
        }
        if (params.length > 0) {
            touched.add(params[0].toString());
        }
        sketch.add(new Cmd(codec, command, params, mainPromise));
    }

    @Override
    public Future<List<?>> executeAsync() {
        RedisException last = null;
        int i = 0;
        while (i < sketch.size()) {
            String kind = sketch.get(i).command.getName();
            int j = i + 1;
            while (j < sketch.size() && sketch.get(j).command.getName().equals(kind) && runnable(kind)) {
                j++;
            }
            try {
                runBatch(sketch.subList(i, j));
            } catch (RedisException e) {
                last = e;
                for (Cmd c : sketch.subList(i, j)) {
                    c.promise.tryFailure(e);
                }
            }
            i = j;
        }
        if (last != null) {
            Promise<List<?>> p = getConnectionManager().newPromise();
            p.setFailure(last);
            return p;
        }
        return super.executeAsync(); // gathers every promise (sketch ones are complete) in index order
    }

    static boolean runnable(String kind) {
        return "PFADD".equals(kind) || "GETBIT".equals(kind) || "SETBIT".equals(kind) || "PFCOUNT".equals(kind);
    }

    void runBatch(List<Cmd> run) {
        String kind = run.get(0).command.getName();
        if (!runnable(kind) || run.size() == 1) {
            for (Cmd c : run) {
                Object reply = GpuSketchCommandService.KEY_COMMANDS.contains(c.command.getName())
                        ? SketchDispatch.keyCommand(ctx, c.codec, c.command, c.params)
                        : SketchDispatch.single(ctx, c.codec, c.command, c.params);
                c.promise.setSuccess(GpuSketchCommandService.convert(c.command, reply));
            }
            return;
        }
        try {
            List<byte[]> keys = new ArrayList<byte[]>();
            for (Cmd c : run) {
                keys.add(GpuSketchCommandService.encodeParam(c.codec, c.command, c.params[0], 1));
            }
            SketchDispatch.Packed k = new SketchDispatch.Packed(keys);
            int n = run.size();
            byte[] out = new byte[n];
            if ("PFADD".equals(kind)) {
                List<byte[]> elems = new ArrayList<byte[]>();
                int[] counts = new int[n];
                for (int c = 0; c < n; c++) {
                    Cmd cmd = run.get(c);
                    counts[c] = cmd.params.length - 1;
                    for (int p = 1; p < cmd.params.length; p++) {
                        elems.add(GpuSketchCommandService.encodeParam(cmd.codec, cmd.command, cmd.params[p], p + 1));
                    }
                }
                SketchDispatch.Packed e = new SketchDispatch.Packed(elems);
                SketchDispatch.pfaddRun(ctx, keys, k, counts, e, out);
            } else if ("PFCOUNT".equals(kind)) {
                for (Cmd c : run) {
                    c.promise.setSuccess(GpuSketchCommandService.convert(c.command,
                            SketchDispatch.single(ctx, c.codec, c.command, c.params)));
                }
                return;
            } else {
                long[] offs = new long[n];
                byte[] vals = new byte[n];
                for (int c = 0; c < n; c++) {
                    offs[c] = Long.parseLong(run.get(c).params[1].toString());
                    if ("SETBIT".equals(kind)) {
                        vals[c] = (byte) Integer.parseInt(run.get(c).params[2].toString());
                    }
                }
                SketchDispatch.check(ctx, "SETBIT".equals(kind)
                        ? SketchNative.setbit(ctx, k.off, k.bytes, offs, vals, out)
                        : SketchNative.getbit(ctx, k.off, k.bytes, offs, out));
            }
            for (int c = 0; c < n; c++) {
                Cmd cmd = run.get(c);
                cmd.promise.setSuccess(GpuSketchCommandService.convert(cmd.command, Long.valueOf(out[c])));
            }
        } catch (RedisException e) {
            throw e;
        } catch (Exception e) {
            throw new RedisException(e.getMessage(), e);
        }
    }
}

/*
 * GpuSketchBatchService -- RBatch executor for sketch commands.
 *
 * CommandBatchService queues (BatchCommandData) per slot with a global index
 * (M:command/CommandBatchService.java:91-111) and answers in enqueue order
 * (:163-171).  This subclass executes the sketch commands of the batch on the
 * GPU instead: the queue is replayed in enqueue order, consecutive commands of
 * the same kind (PFADD / GETBIT / SETBIT / PFCOUNT) become ONE device batch
 * (exact sequential replies inside the batch, sk_pfadd / sk_setbit /
 * sk_pfcount).  The batch's other commands still go to redis-server through
 * super.executeAsync(), even when a sketch command failed, as the reference
 * pipeline executes every command (:142-182).  The result list holds every
 * command's reply in enqueue order, sketch and redis alike; if any command
 * failed the future fails with the error of the last failed command in that
 * order, as CommandDecoder does (M:client/handler/CommandDecoder.java:183-197).
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
import org.redisson.client.protocol.RedisCommands;
import org.redisson.client.protocol.convertor.VoidReplayConvertor;
import org.redisson.command.CommandBatchService;
import org.redisson.connection.ConnectionManager;
import org.redisson.connection.NodeSource;

import io.netty.util.concurrent.Future;
import io.netty.util.concurrent.FutureListener;
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
    final List<Promise<?>> order = new ArrayList<Promise<?>>(); // every command's promise, enqueue order
    final Set<String> touched = new HashSet<String>();
    boolean redisUsed;
    boolean executed;

    public GpuSketchBatchService(ConnectionManager connectionManager, long ctx) {
        super(connectionManager);
        this.ctx = ctx;
    }

    @Override
    protected <V, R> void async(boolean readOnlyMode, NodeSource nodeSource, Codec codec, RedisCommand<V> command,
                                Object[] params, Promise<R> mainPromise, int attempt) {
        if (executed) {
            throw new IllegalStateException("Batch already has been executed!");
        }
        order.add(mainPromise);
        String name = command.getName();
        if ("DEL".equals(name) && params.length > 0) {
            delAsync(readOnlyMode, nodeSource, codec, command, params, mainPromise, attempt);
            return;
        }
        // GET / SET join the sketch queue when the engine holds the key, or an earlier sketch command of this
        // batch names it (it may create the key before this one runs)
        boolean keyCommand = GpuSketchCommandService.KEY_COMMANDS.contains(name) && params.length > 0
                && (touched.contains(params[0].toString()) || SketchDispatch.engineHolds(ctx, params[0]));
        if (!keyCommand && !GpuSketchCommandService.SKETCH_COMMANDS.contains(name)) {
            redisUsed = true;
            super.async(readOnlyMode, nodeSource, codec, command, params, mainPromise, attempt);
            return;
        }
        if (params.length > 0) {
            touched.add(params[0].toString());
        }
        sketch.add(new Cmd(codec, command, params, mainPromise));
    }

    /* DEL inside a batch, split by holder: the engine part runs in the sketch queue at the command's place, the
     * redis part joins the redis batch; the command's promise gets the sum once both are done. */
    @SuppressWarnings({"unchecked", "rawtypes"})
    <V, R> void delAsync(boolean readOnlyMode, NodeSource nodeSource, Codec codec, final RedisCommand<V> command,
                         Object[] params, final Promise<R> mainPromise, int attempt) {
        List<Object>[] parts = SketchDispatch.splitDel(ctx, params, touched);
        if (parts[0].isEmpty()) {
            redisUsed = true;
            super.async(readOnlyMode, nodeSource, codec, command, params, mainPromise, attempt);
            return;
        }
        if (parts[1].isEmpty()) {
            sketch.add(new Cmd(codec, command, params, mainPromise));
            return;
        }
        final Promise<Object> engine = getConnectionManager().newPromise();
        final Promise<Object> redis = getConnectionManager().newPromise();
        FutureListener<Object> both = new FutureListener<Object>() {
            @Override
            public void operationComplete(Future<Object> f) throws Exception {
                if (!engine.isDone() || !redis.isDone()) {
                    return;
                }
                if (!engine.isSuccess()) {
                    mainPromise.tryFailure(engine.cause());
                } else if (!redis.isSuccess()) {
                    mainPromise.tryFailure(redis.cause());
                } else {
                    long n = ((Number) engine.getNow()).longValue() + ((Number) redis.getNow()).longValue();
                    mainPromise.trySuccess((R) GpuSketchCommandService.convert(command, Long.valueOf(n)));
                }
            }
        };
        engine.addListener(both);
        redis.addListener(both);
        sketch.add(new Cmd(codec, RedisCommands.DEL, parts[0].toArray(), engine));
        redisUsed = true;
        super.async(readOnlyMode, nodeSource, codec, RedisCommands.DEL, parts[1].toArray(), (Promise) redis, attempt);
    }

    @Override
    public Future<List<?>> executeAsync() {
        if (executed) {
            throw new IllegalStateException("Batch already executed!");
        }
        if (order.isEmpty()) {
            return getConnectionManager().newSucceededFuture(null);
        }
        executed = true;
        final Promise<List<?>> result = getConnectionManager().newPromise();
        final GpuBatchCoalescer co = GpuBatchCoalescer.of(ctx);
        // the sketch runs and the hand-off of the redis part happen on the context's worker: the caller (maybe an
        // event-loop thread) never waits on the device
        try {
            if (co != null && pfaddOnly()) { // group commit with the PFADD-only batches queued beside it
                submitGroup(co, result);
                return result;
            }
            Runnable task = new Runnable() {
                @Override
                public void run() {
                    try {
                        executeOnWorker(result);
                    } catch (RuntimeException e) {
                        result.tryFailure(e);
                    }
                }
            };
            if (co != null) {
                co.executeAfter(task);
            } else {
                SketchDispatch.worker(ctx).execute(task);
            }
        } catch (java.util.concurrent.RejectedExecutionException e) {
            result.tryFailure(new IllegalStateException("sketch engine shut down", e));
        }
        return result;
    }

    /* RBitSet range set/clear (M:RedissonBitSet.java:202-228) and RedissonBloomFilter's pipelines finish their
     * batch with executeAsyncVoid, which in the reference walks the per-slot queues directly
     * (M:command/CommandBatchService.java:117-140) and would never see this class's sketch queue: route it through
     * executeAsync and drop the result list. */
    @Override
    public Future<Void> executeAsyncVoid() {
        final Promise<Void> done = getConnectionManager().newPromise();
        executeAsync().addListener(new FutureListener<List<?>>() {
            @Override
            public void operationComplete(Future<List<?>> f) throws Exception {
                if (f.isSuccess()) {
                    done.trySuccess(null);
                } else {
                    done.tryFailure(f.cause());
                }
            }
        });
        return done;
    }

    boolean pfaddOnly() {
        if (redisUsed || sketch.isEmpty()) {
            return false;
        }
        for (Cmd c : sketch) {
            if (!"PFADD".equals(c.command.getName())) {
                return false;
            }
        }
        return true;
    }

    /* the batch as one request of the context's GpuBatchCoalescer: its commands' encoded keys and elements; the
     * group's replies complete the command promises and the batch result in enqueue order */
    void submitGroup(GpuBatchCoalescer co, final Promise<List<?>> result) {
        List<byte[]> keys = new ArrayList<byte[]>(sketch.size());
        List<byte[][]> elems = new ArrayList<byte[][]>(sketch.size());
        for (Cmd c : sketch) {
            keys.add(GpuSketchCommandService.encodeParam(c.codec, c.command, c.params[0], 1));
            byte[][] es = new byte[c.params.length - 1][];
            for (int p = 1; p < c.params.length; p++) {
                es[p - 1] = GpuSketchCommandService.encodeParam(c.codec, c.command, c.params[p], p + 1);
            }
            elems.add(es);
        }
        Promise<boolean[]> replies = getConnectionManager().newPromise();
        replies.addListener(new FutureListener<boolean[]>() {
            @Override
            public void operationComplete(Future<boolean[]> f) throws Exception {
                if (!f.isSuccess()) {
                    for (Cmd c : sketch) {
                        c.promise.tryFailure(f.cause());
                    }
                    result.tryFailure(f.cause());
                    return;
                }
                boolean[] rep = f.getNow();
                List<Object> out = new ArrayList<Object>(sketch.size());
                for (int i = 0; i < rep.length; i++) {
                    Cmd c = sketch.get(i);
                    c.promise.trySuccess(GpuSketchCommandService.convert(c.command, Long.valueOf(rep[i] ? 1 : 0)));
                    out.add(c.promise.getNow());
                }
                result.trySuccess(out);
            }
        });
        co.submit(keys, elems, replies);
    }

    void executeOnWorker(final Promise<List<?>> result) {
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
                for (Cmd c : sketch.subList(i, j)) {
                    c.promise.tryFailure(e);
                }
            }
            i = j;
        }
        // the redis-side commands are sent whatever happened above (the reference pipeline executes them all)
        Future<List<?>> redis = redisUsed ? super.executeAsync()
                : getConnectionManager().<List<?>>newSucceededFuture(null);
        redis.addListener(new FutureListener<List<?>>() {
            @Override
            public void operationComplete(Future<List<?>> f) throws Exception {
                Throwable last = null;
                List<Object> out = new ArrayList<Object>(order.size());
                for (Promise<?> p : order) {
                    if (!p.isDone()) { // a redis command the failed batch never answered
                        last = f.isSuccess() ? new RedisException("batch command not executed") : f.cause();
                        out.add(null);
                        continue;
                    }
                    if (!p.isSuccess()) {
                        last = p.cause();
                    }
                    out.add(p.getNow());
                }
                if (last == null && !f.isSuccess()) {
                    last = f.cause();
                }
                if (last != null) {
                    result.setFailure(last);
                } else {
                    result.setSuccess(out);
                }
            }
        });
    }

    /* A run of SETBIT_VOID on one key, one value and consecutive offsets -- what RBitSet.set(from, to) and
     * clear(from, to) queue, one SETBIT per bit (M:RedissonBitSet.java:202-228) -- is applied by ONE range kernel
     * with the same string growth and final bits (k_bit_range).  The replies are Void, so nothing else is owed;
     * an out-of-range offset fails the run after the in-range bits are set, as the pipeline would. */
    boolean bitRange(List<Cmd> run) {
        if (run.size() < 64) {
            return false;
        }
        Cmd first = run.get(0);
        String key = first.params[0].toString();
        String val = first.params[2].toString();
        long from = Long.parseLong(first.params[1].toString());
        for (int c = 0; c < run.size(); c++) {
            Cmd cmd = run.get(c);
            if (!(cmd.command.getConvertor() instanceof VoidReplayConvertor) || !key.equals(cmd.params[0].toString())
                    || !val.equals(cmd.params[2].toString())
                    || Long.parseLong(cmd.params[1].toString()) != from + c) {
                return false;
            }
        }
        byte[] k = GpuSketchCommandService.encodeParam(first.codec, first.command, first.params[0], 1);
        SketchDispatch.check(ctx, SketchNative.setBitRange(ctx, k, from, from + run.size(), !"0".equals(val)));
        for (Cmd cmd : run) {
            cmd.promise.setSuccess(null);
        }
        return true;
    }

    static boolean runnable(String kind) {
        return "PFADD".equals(kind) || "GETBIT".equals(kind) || "SETBIT".equals(kind) || "PFCOUNT".equals(kind);
    }

    void runBatch(List<Cmd> run) {
        String kind = run.get(0).command.getName();
        if (!runnable(kind) || run.size() == 1) {
            for (Cmd c : run) {
                try {
                    Object reply = GpuSketchCommandService.KEY_COMMANDS.contains(c.command.getName())
                            ? SketchDispatch.keyCommand(ctx, c.codec, c.command, c.params)
                            : SketchDispatch.single(ctx, c.codec, c.command, c.params);
                    c.promise.setSuccess(GpuSketchCommandService.convert(c.command, reply));
                } catch (RedisException e) { // this command alone fails (pipeline semantics)
                    c.promise.tryFailure(e);
                }
            }
            return;
        }
        try {
            int n = run.size();
            if ("PFCOUNT".equals(kind)) { // one sk_pfcount for the run
                List<RedisCommand<?>> cmds = new ArrayList<RedisCommand<?>>();
                List<Object[]> params = new ArrayList<Object[]>();
                for (Cmd c : run) {
                    cmds.add(c.command);
                    params.add(c.params);
                }
                long[] counts = SketchDispatch.pfcountRun(ctx, run.get(0).codec, cmds, params);
                for (int c = 0; c < n; c++) {
                    run.get(c).promise.setSuccess(GpuSketchCommandService.convert(run.get(c).command,
                            Long.valueOf(counts[c])));
                }
                return;
            }
            List<byte[]> keys = new ArrayList<byte[]>();
            for (Cmd c : run) {
                keys.add(GpuSketchCommandService.encodeParam(c.codec, c.command, c.params[0], 1));
            }
            SketchDispatch.Packed k = new SketchDispatch.Packed(keys);
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
            } else if ("SETBIT".equals(kind) && bitRange(run)) {
                return; // one range kernel (sk_set_bit_range) for the whole run
            } else {
                long[] offs = new long[n];
                byte[] vals = new byte[n];
                for (int c = 0; c < n; c++) {
                    offs[c] = Long.parseLong(run.get(c).params[1].toString());
                    if ("SETBIT".equals(kind)) {
                        vals[c] = (byte) Integer.parseInt(run.get(c).params[2].toString());
                    }
                }
                // SETBIT_VOID (RBitSet.set(i), M:RedissonBitSet.java:79-81) owes no reply: a null reply array lets
                // the engine take the SETBIT_VOID kernels (sk_setbit, the dense region path for dense runs)
                boolean allVoid = true;
                for (Cmd c : run) {
                    allVoid &= c.command == RedisCommands.SETBIT_VOID;
                }
                SketchDispatch.check(ctx, "SETBIT".equals(kind)
                        ? SketchNative.setbit(ctx, k.off, k.bytes, offs, vals, allVoid ? null : out)
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

/*
 * SketchRouter -- the engine routing every L3 executor of the integration shares.
 *
 * The reference has three executor families over one hook, CommandAsyncService.async(readOnly, NodeSource, Codec,
 * RedisCommand, Object[] params, Promise, attempt) (M:command/CommandAsyncService.java:378):
 *   Redisson          -> CommandSyncService     (M:Redisson.java:118)
 *   RedissonReactive  -> CommandReactiveService (M:RedissonReactive.java:106, M:command/CommandReactiveService.java:35)
 *   RBatch / RBatchReactive / internal batches -> CommandBatchService (M:RedissonBatch.java:61,
 *                        M:reactive/RedissonBatchReactive.java:51, M:RedissonBitSet.java:204,223)
 * GpuSketchCommandService and GpuSketchReactiveService subclass the first two and send their async() here;
 * GpuSketchBatchService subclasses the third.  A command whose name is a sketch command -- or a GET / SET / DEL /
 * RBitSet.length() EVAL on a key the engine holds -- runs on the engine, on the context's FIFO worker
 * (SketchDispatch.worker: no caller thread, which may be a Netty event loop, waits on the device); everything else
 * goes to redis-server through the executor's own super.async (RedisPath).  Source only here; see INTEGRATION.md.
 */
package org.redisson.gpu;

import java.security.MessageDigest;
import java.util.List;
import java.util.concurrent.RejectedExecutionException;

import org.redisson.client.RedisException;
import org.redisson.client.codec.Codec;
import org.redisson.client.protocol.RedisCommand;
import org.redisson.client.protocol.RedisCommands;
import org.redisson.connection.ConnectionManager;
import org.redisson.connection.NodeSource;

import io.netty.util.concurrent.Future;
import io.netty.util.concurrent.FutureListener;
import io.netty.util.concurrent.Promise;

public final class SketchRouter {
    private SketchRouter() {
    }

    /** The executor's own path to redis-server: its super.async (CommandSyncService / CommandReactiveService). */
    public interface RedisPath {
        <V, R> void redisAsync(boolean readOnlyMode, NodeSource source, Codec codec, RedisCommand<V> command,
                               Object[] params, Promise<R> mainPromise, int attempt);

        ConnectionManager getConnectionManager();
    }

    /* RBitSet.lengthAsync's Lua script (M:RedissonBitSet.java:181-191), recognised by the SHA1 of its body as the
     * RESP front-end does (sk_resp.cpp kScriptBitsetLength; tools/script_digests.py derives it). */
    static final String LENGTH_SCRIPT_SHA1 = "a80ae5bc82f0ec7382e36b49cdc6bc589a9a80b3";

    static boolean isLengthScript(RedisCommand<?> command, Object[] params) {
        if (!"EVAL".equals(command.getName()) || params.length != 3 || !(params[0] instanceof String)
                || !"1".equals(String.valueOf(params[1]))) {
            return false;
        }
        try {
            byte[] d = MessageDigest.getInstance("SHA-1").digest(((String) params[0]).getBytes(GpuSketchCommandService.UTF8));
            StringBuilder hex = new StringBuilder(40);
            for (byte b : d) {
                hex.append(String.format("%02x", b & 0xff));
            }
            return LENGTH_SCRIPT_SHA1.equals(hex.toString());
        } catch (java.security.NoSuchAlgorithmException e) {
            return false;
        }
    }

    /** Whether the command may belong to the engine; the rest never leaves the caller's thread. */
    static boolean candidate(RedisCommand<?> command) {
        String name = command.getName();
        return GpuSketchCommandService.SKETCH_COMMANDS.contains(name)
                || GpuSketchCommandService.KEY_COMMANDS.contains(name) || "FLUSHALL".equals(name)
                || "EVAL".equals(name);
    }

    /**
     * The executor's async(): returns false when the command is redis-server's (the caller then calls its own
     * super.async at once); otherwise the engine work is queued on the context's worker and true is returned.
     */
    public static <V, R> boolean submit(final long ctx, final RedisPath redis, final boolean readOnlyMode,
                                        final NodeSource source, final Codec codec, final RedisCommand<V> command,
                                        final Object[] params, final Promise<R> mainPromise, final int attempt) {
        if (!candidate(command) || ("EVAL".equals(command.getName()) && !isLengthScript(command, params))) {
            return false;
        }
        try {
            SketchDispatch.worker(ctx).execute(new Runnable() {
                @Override
                public void run() {
                    try {
                        onWorker(ctx, redis, readOnlyMode, source, codec, command, params, mainPromise, attempt);
                    } catch (RuntimeException e) {
                        mainPromise.tryFailure(e);
                    }
                }
            });
        } catch (RejectedExecutionException e) {
            mainPromise.tryFailure(new IllegalStateException("sketch engine shut down", e));
        }
        return true;
    }

    /* on the worker thread */
    static <V, R> void onWorker(long ctx, RedisPath redis, boolean readOnlyMode, NodeSource source, Codec codec,
                                RedisCommand<V> command, Object[] params, Promise<R> mainPromise, int attempt) {
        String name = command.getName();
        if ("FLUSHALL".equals(name)) { // both stores; every cached slab handle is dead
            SketchDispatch.invalidateAll(ctx);
            SketchDispatch.check(ctx, SketchNative.flushall(ctx));
            redis.redisAsync(readOnlyMode, source, codec, command, params, mainPromise, attempt);
            return;
        }
        if ("DEL".equals(name) && params.length > 0) {
            del(ctx, redis, readOnlyMode, source, codec, command, params, mainPromise, attempt);
            return;
        }
        if ("EVAL".equals(name)) { // RBitSet.length() of an engine bitset: BITPOS + GETBIT walk on the device
            if (!SketchDispatch.engineHolds(ctx, params[2])) {
                redis.redisAsync(readOnlyMode, source, codec, command, params, mainPromise, attempt);
                return;
            }
            try {
                long[] out = new long[1];
                SketchDispatch.check(ctx, SketchNative.bitsetLength(ctx, SketchDispatch.keyBytes(params[2]), out));
                @SuppressWarnings("unchecked")
                R r = (R) GpuSketchCommandService.convert(command, Long.valueOf(out[0]));
                mainPromise.setSuccess(r);
            } catch (RedisException e) {
                mainPromise.setFailure(e);
            }
            return;
        }
        boolean keyCommand = GpuSketchCommandService.KEY_COMMANDS.contains(name) && params.length > 0
                && SketchDispatch.engineHolds(ctx, params[0]);
        if (!keyCommand && !GpuSketchCommandService.SKETCH_COMMANDS.contains(name)) {
            redis.redisAsync(readOnlyMode, source, codec, command, params, mainPromise, attempt);
            return;
        }
        try {
            Object reply = keyCommand ? SketchDispatch.keyCommand(ctx, codec, command, params)
                    : SketchDispatch.single(ctx, codec, command, params);
            @SuppressWarnings("unchecked")
            R r = (R) GpuSketchCommandService.convert(command, reply);
            mainPromise.setSuccess(r);
        } catch (RedisException e) {
            mainPromise.setFailure(e);
        }
    }

    /* DEL k1..kn: engine-held keys are deleted on the engine, the others on redis-server (ADVICE r1: RBloomFilter
     * .delete sends DEL name {name}__config, M:RedissonBloomFilter.java:201-203); the reply is the sum of both
     * counts through the command's own convertor (DEL, DEL_BOOL, DEL_OBJECTS, DEL_VOID). */
    @SuppressWarnings("unchecked")
    static <V, R> void del(long ctx, RedisPath redis, boolean readOnlyMode, NodeSource source, Codec codec,
                           final RedisCommand<V> command, Object[] params, final Promise<R> mainPromise,
                           int attempt) {
        List<Object>[] parts = SketchDispatch.splitDel(ctx, params, null);
        if (parts[0].isEmpty()) {
            redis.redisAsync(readOnlyMode, source, codec, command, params, mainPromise, attempt);
            return;
        }
        final long engineCount;
        try {
            engineCount = ((Long) SketchDispatch.keyCommand(ctx, codec, RedisCommands.DEL, parts[0].toArray()))
                    .longValue();
        } catch (RedisException e) {
            mainPromise.setFailure(e);
            return;
        }
        if (parts[1].isEmpty()) {
            mainPromise.setSuccess((R) GpuSketchCommandService.convert(command, Long.valueOf(engineCount)));
            return;
        }
        Promise<Long> rest = redis.getConnectionManager().newPromise();
        rest.addListener(new FutureListener<Long>() {
            @Override
            public void operationComplete(Future<Long> f) throws Exception {
                if (!f.isSuccess()) {
                    mainPromise.setFailure(f.cause());
                    return;
                }
                mainPromise.setSuccess((R) GpuSketchCommandService.convert(command,
                        Long.valueOf(engineCount + f.getNow().longValue())));
            }
        });
        redis.redisAsync(readOnlyMode, source, codec, RedisCommands.DEL, parts[1].toArray(), rest, attempt);
    }
}

/*
 * GpuSketchCommandService -- Redisson L3 executor that serves the
 * probabilistic-structure commands from the MI355X sketch engine.
 *
 * Plugs in at the seam the reference already has: CommandAsyncService.async(...)
 * (M:command/CommandAsyncService.java:378) is the single hook every
 * writeAsync/readAsync goes through; CommandBatchService overrides the same
 * hook to queue (M:command/CommandBatchService.java:91).  Commands whose name
 * is a sketch command are executed through JNI; everything else falls through
 * to the Netty -> redis-server path unchanged.  Interfaces in core/ and api/
 * (RHyperLogLog, RBitSet, RBloomFilter, RBatch) are untouched.
 *
 * Source only here (no JDK in the build image); see INTEGRATION.md.
 */
package org.redisson.gpu;

import java.nio.charset.Charset;
import java.util.Arrays;
import java.util.HashSet;
import java.util.List;
import java.util.Set;
import java.util.concurrent.RejectedExecutionException;

import org.redisson.client.RedisException;
import org.redisson.client.codec.Codec;
import org.redisson.client.codec.StringCodec;
import org.redisson.client.protocol.DefaultParamsEncoder;
import org.redisson.client.protocol.Encoder;
import org.redisson.client.protocol.RedisCommand;
import org.redisson.client.protocol.RedisCommand.ValueType;
import org.redisson.client.protocol.RedisCommands;
import org.redisson.command.CommandAsyncService;
import org.redisson.connection.ConnectionManager;
import org.redisson.connection.NodeSource;

import io.netty.util.concurrent.Future;
import io.netty.util.concurrent.FutureListener;
import io.netty.util.concurrent.Promise;

public class GpuSketchCommandService extends CommandAsyncService {

    static final Set<String> SKETCH_COMMANDS = new HashSet<String>(Arrays.asList(
            "PFADD", "PFCOUNT", "PFMERGE", "SETBIT", "GETBIT", "BITCOUNT", "BITOP", "STRLEN"));
    static final Charset UTF8 = Charset.forName("UTF-8");
    /* Generic key commands that act on a sketch key when the engine holds it: RBitSet.toByteArray (GET,
     * M:RedissonBitSet.java:88-91), set(BitSet) (SET, :211-214), clear() / delete() (DEL, :250-253).  The same
     * commands on keys the engine does not hold (RBucket ...) still go to redis-server; DEL is split by holder. */
    static final Set<String> KEY_COMMANDS = new HashSet<String>(Arrays.asList("GET", "SET", "DEL"));
    static final Encoder PARAMS = new DefaultParamsEncoder();

    final long ctx;
    /* Engine work never runs on the caller's thread (often a Netty event-loop thread, SURVEY 8b): the context's
     * FIFO worker (SketchDispatch.worker) makes the JNI calls -- which may wait on the device -- and completes the
     * promises, so the engine sees one caller's commands in the order they were issued.  Commands for redis-server
     * are handed to the reference path at once, or from the worker once it knows the engine does not hold the
     * key. */
    public GpuSketchCommandService(ConnectionManager connectionManager, long ctx) {
        super(connectionManager);
        this.ctx = ctx;
    }

    @Override
    protected <V, R> void async(final boolean readOnlyMode, final NodeSource source, final Codec codec,
                                final RedisCommand<V> command, final Object[] params, final Promise<R> mainPromise,
                                final int attempt) {
        String name = command.getName();
        if (!SKETCH_COMMANDS.contains(name) && !KEY_COMMANDS.contains(name) && !"FLUSHALL".equals(name)) {
            super.async(readOnlyMode, source, codec, command, params, mainPromise, attempt);
            return;
        }
        try {
            SketchDispatch.worker(ctx).execute(new Runnable() {
                @Override
                public void run() {
                    try {
                        engineAsync(readOnlyMode, source, codec, command, params, mainPromise, attempt);
                    } catch (RuntimeException e) {
                        mainPromise.tryFailure(e);
                    }
                }
            });
        } catch (RejectedExecutionException e) {
            mainPromise.tryFailure(new IllegalStateException("sketch engine shut down", e));
        }
    }

    /* on the worker thread */
    <V, R> void engineAsync(boolean readOnlyMode, NodeSource source, Codec codec, RedisCommand<V> command,
                            Object[] params, Promise<R> mainPromise, int attempt) {
        String name = command.getName();
        if ("FLUSHALL".equals(name)) { // both stores; every cached slab handle is dead
            SketchDispatch.invalidateAll(ctx);
            SketchDispatch.check(ctx, SketchNative.flushall(ctx));
            super.async(readOnlyMode, source, codec, command, params, mainPromise, attempt);
            return;
        }
        if ("DEL".equals(name) && params.length > 0) {
            del(readOnlyMode, source, codec, command, params, mainPromise, attempt);
            return;
        }
        boolean keyCommand = KEY_COMMANDS.contains(name) && params.length > 0
                && SketchDispatch.engineHolds(ctx, params[0]);
        if (!keyCommand && !SKETCH_COMMANDS.contains(name)) {
            super.async(readOnlyMode, source, codec, command, params, mainPromise, attempt);
            return;
        }
        try {
            Object reply = keyCommand ? SketchDispatch.keyCommand(ctx, codec, command, params)
                    : SketchDispatch.single(ctx, codec, command, params);
            @SuppressWarnings("unchecked")
            R r = (R) convert(command, reply);
            mainPromise.setSuccess(r);
        } catch (RedisException e) {
            mainPromise.setFailure(e);
        }
    }

    /* DEL k1..kn: engine-held keys are deleted on the engine, the others on redis-server (ADVICE r1: RBloomFilter
     * .delete sends DEL name {name}__config, M:RedissonBloomFilter.java:201-203); the reply is the sum of both
     * counts through the command's own convertor (DEL, DEL_BOOL, DEL_OBJECTS, DEL_VOID). */
    @SuppressWarnings({"unchecked", "rawtypes"})
    <V, R> void del(boolean readOnlyMode, NodeSource source, Codec codec, final RedisCommand<V> command,
                    Object[] params, final Promise<R> mainPromise, int attempt) {
        List<Object>[] parts = SketchDispatch.splitDel(ctx, params, null);
        if (parts[0].isEmpty()) {
            super.async(readOnlyMode, source, codec, command, params, mainPromise, attempt);
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
            mainPromise.setSuccess((R) convert(command, Long.valueOf(engineCount)));
            return;
        }
        Promise<Long> redis = getConnectionManager().newPromise();
        redis.addListener(new FutureListener<Long>() {
            @Override
            public void operationComplete(Future<Long> f) throws Exception {
                if (!f.isSuccess()) {
                    mainPromise.setFailure(f.cause());
                    return;
                }
                mainPromise.setSuccess((R) convert(command, Long.valueOf(engineCount + f.getNow().longValue())));
            }
        });
        super.async(readOnlyMode, source, codec, RedisCommands.DEL, parts[1].toArray(), redis, attempt);
    }

    /** The reply convertor the RedisCommand carries (BooleanReplayConvertor, BitSetReplayConvertor ...). */
    static Object convert(RedisCommand<?> command, Object reply) {
        if (command.getConvertor() == null || reply == null) {
            return reply;
        }
        return command.getConvertor().convert(reply);
    }

    /**
     * CommandEncoder.encode's choice of encoder for param i (1-based), M:client/handler/CommandEncoder.java:73-94:
     * with one in-param type, the param AT inParamIndex goes through the codec's value encoder when the type is
     * OBJECT, and params from inParamIndex on go through selectEncoder when it is not; with several types, every
     * param from inParamIndex on goes through selectEncoder(i - inParamIndex); the rest use DefaultParamsEncoder
     * (byte[] as is, else toString() UTF-8).
     */
    static byte[] encodeParam(Codec codec, RedisCommand<?> command, Object param, int i) throws Exception {
        Encoder encoder = PARAMS;
        List<ValueType> types = command.getInParamType();
        int idx = command.getInParamIndex();
        if (types.size() == 1) {
            if (idx == i && types.get(0) == ValueType.OBJECT) {
                encoder = codec.getValueEncoder();
            } else if (idx <= i && types.get(0) != ValueType.OBJECT) {
                encoder = selectEncoder(codec, types, i - idx);
            }
        } else if (idx <= i) {
            encoder = selectEncoder(codec, types, i - idx);
        }
        return encoder.encode(param);
    }

    /** CommandEncoder.selectEncoder, M:client/handler/CommandEncoder.java:101-130. */
    static Encoder selectEncoder(Codec codec, List<ValueType> types, int param) {
        int typeIndex = types.size() > 1 ? param : 0;
        ValueType t = types.get(typeIndex);
        if (t == ValueType.MAP) {
            return param % 2 != 0 ? codec.getMapValueEncoder() : codec.getMapKeyEncoder();
        }
        if (t == ValueType.MAP_KEY) {
            return codec.getMapKeyEncoder();
        }
        if (t == ValueType.MAP_VALUE) {
            return codec.getMapValueEncoder();
        }
        if (t == ValueType.OBJECTS || t == ValueType.OBJECT) {
            return codec.getValueEncoder();
        }
        if (t == ValueType.STRING) {
            return StringCodec.INSTANCE.getValueEncoder();
        }
        throw new IllegalStateException();
    }
}

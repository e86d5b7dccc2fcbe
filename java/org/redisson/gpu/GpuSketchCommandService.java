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
import java.util.Set;

import org.redisson.client.RedisException;
import org.redisson.client.codec.Codec;
import org.redisson.client.protocol.RedisCommand;
import org.redisson.client.protocol.RedisCommand.ValueType;
import org.redisson.command.CommandAsyncService;
import org.redisson.connection.ConnectionManager;
import org.redisson.connection.NodeSource;

import io.netty.util.concurrent.Promise;

public class GpuSketchCommandService extends CommandAsyncService {

    static final Set<String> SKETCH_COMMANDS = new HashSet<String>(Arrays.asList(
            "PFADD", "PFCOUNT", "PFMERGE", "SETBIT", "GETBIT", "BITCOUNT", "BITOP", "STRLEN"));
    static final Charset UTF8 = Charset.forName("UTF-8");
    /* Generic key commands that act on a sketch key when the engine holds it: RBitSet.toByteArray (GET,
     * M:RedissonBitSet.java:88-91), set(BitSet) (SET, :211-214), clear() / delete() (DEL, :250-253).  The same
     * commands on keys the engine does not hold (RBucket ...) still go to redis-server. */
    static final Set<String> KEY_COMMANDS = new HashSet<String>(Arrays.asList("GET", "SET", "DEL"));

    final long ctx;

    public GpuSketchCommandService(ConnectionManager connectionManager, long ctx) {
        super(connectionManager);
        this.ctx = ctx;
    }

    @Override
    protected <V, R> void async(boolean readOnlyMode, NodeSource source, Codec codec, RedisCommand<V> command,
                                Object[] params, Promise<R> mainPromise, int attempt) {
        boolean keyCommand = KEY_COMMANDS.contains(command.getName()) && params.length > 0
                && SketchDispatch.engineHolds(ctx, params[0]);
        if (!keyCommand && !SKETCH_COMMANDS.contains(command.getName())) {
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

    /** The reply convertor the RedisCommand carries (BooleanReplayConvertor, BitSetReplayConvertor ...). */
    static Object convert(RedisCommand<?> command, Object reply) {
        if (command.getConvertor() == null || reply == null) {
            return reply;
        }
        return command.getConvertor().convert(reply);
    }

    /**
     * CommandEncoder param rules (M:client/handler/CommandEncoder.java:73-94): the
     * param at inParamIndex with OBJECT type goes through the codec's value encoder;
     * the rest are DefaultParamsEncoder (byte[] raw, else toString() UTF-8).
     */
    static byte[] encodeParam(Codec codec, RedisCommand<?> command, Object param, int i) throws Exception {
        if (command.getInParamType().size() == 1 && command.getInParamIndex() == i
                && command.getInParamType().get(0) == ValueType.OBJECT) {
            return codec.getValueEncoder().encode(param);
        }
        if (param instanceof byte[]) {
            return (byte[]) param;
        }
        return param.toString().getBytes(UTF8);
    }
}

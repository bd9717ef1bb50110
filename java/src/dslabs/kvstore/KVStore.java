package dslabs.kvstore;

import dslabs.framework.Application;
import dslabs.framework.Command;
import dslabs.framework.Result;
import java.util.HashMap;
import java.util.Map;
import lombok.Data;
import lombok.EqualsAndHashCode;
import lombok.NonNull;
import lombok.ToString;

/**
 * The lab1 key-value store (DESIGN.md §11): Get -> GetResult(value) or KeyNotFound, Put -> PutOk,
 * Append -> AppendResult(new value), as KVStoreWorkload expects (KVStoreWorkload.java:40-66). The
 * command and result types are the reference stub's own declarations
 * (labs/lab1-clientserver/src/dslabs/kvstore/KVStore.java:15-58: Lombok @Data, fluent accessors
 * from the repository's lombok.config), so their equality and toString -- which PaxosTest's
 * hasCommand predicate names carry, "KVStore.Append(key=foo, value=X)" -- are Lombok's; only
 * execute() is written here. On the device a key is a key id (<= 3 keys) and a value a sequence of
 * <= 9 equal-length workload tokens (amokv.hpp).
 */
@ToString
@EqualsAndHashCode
public class KVStore implements Application {

  public interface KVStoreCommand extends Command {}

  public interface SingleKeyCommand extends KVStoreCommand {
    String key();
  }

  @Data
  public static final class Get implements SingleKeyCommand {
    @NonNull private final String key;

    @Override
    public boolean readOnly() {
      return true;
    }
  }

  @Data
  public static final class Put implements SingleKeyCommand {
    @NonNull private final String key, value;
  }

  @Data
  public static final class Append implements SingleKeyCommand {
    @NonNull private final String key, value;
  }

  public interface KVStoreResult extends Result {}

  @Data
  public static final class GetResult implements KVStoreResult {
    @NonNull private final String value;
  }

  @Data
  public static final class KeyNotFound implements KVStoreResult {}

  @Data
  public static final class PutOk implements KVStoreResult {}

  @Data
  public static final class AppendResult implements KVStoreResult {
    @NonNull private final String value;
  }

  private final Map<String, String> data = new HashMap<>();

  @Override
  public KVStoreResult execute(Command command) {
    if (command instanceof Get g) {
      String v = data.get(g.key());
      return v == null ? new KeyNotFound() : new GetResult(v);
    }
    if (command instanceof Put p) {
      data.put(p.key(), p.value());
      return new PutOk();
    }
    if (command instanceof Append a) {
      String v = data.getOrDefault(a.key(), "") + a.value();
      data.put(a.key(), v);
      return new AppendResult(v);
    }
    throw new IllegalArgumentException();
  }
}

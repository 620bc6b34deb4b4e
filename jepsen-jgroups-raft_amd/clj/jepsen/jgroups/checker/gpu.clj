(ns jepsen.jgroups.checker.gpu
  "Drop-in for (checker/linearizable {:model m :algorithm :linear}) backed by
  liblincheck.so (include/lincheck.h) through JNA. Reference call sites replaced:
  src/jepsen/jgroups/workload/register.clj:106-111 (independent/checker over
  checker/linearizable), counter.clj:133-137 (model CounterModel, :100-127) and leader.clj:79-85
  (model (LeaderModel. {}), :63-75).

  UNTESTED ON A JVM: the build container and the GPU box have no JVM, so this file has
  never been loaded. The Python ctypes harness (lincheck/_lib.py, lincheck/checker.py)
  makes the same calls with the same arrays and is what the tests exercise."
  (:require [jepsen.checker :as checker]
            [jepsen.independent :as independent]
            [knossos.model :as model])
  (:import (com.sun.jna NativeLibrary Function)
           (knossos.model CASRegister)))

(def ^:private lib (delay (NativeLibrary/getInstance "lincheck")))

(defn- lib-fn
  "The exported C function `fname` of liblincheck.so."
  ^Function [fname]
  (.getFunction ^NativeLibrary @lib ^String fname))

(def type-code {:invoke 0 :ok 1 :fail 2 :info 3})
(def f-code {:read 0 :write 1 :cas 2 :add 3 :decr 4 :add-and-get 5 :decr-and-get 6 :inspect 7})

(defn- leader-name
  "serialize-leader (leader.clj:51-54): nil -> \"null\"."
  [x]
  (if (nil? x) "null" (str x)))

(def ^:private err-text
  {-4 "malformed history" -5 "too many concurrently pending ops"
   -6 "model cannot step an op" -7 "frontier exceeded max-configs / device capacity"
   -8 "device search aborted by its barrier watchdog (device not wholly available)"})

(defn- c-string [^bytes buf]
  (String. buf 0 (int (or (first (keep-indexed #(when (zero? %2) %1) buf)) (alength buf)))))

(defn- encode
  "Histories (seq of op vectors) -> SoA primitive arrays in lincheck.h order."
  [histories]
  (let [ops    (vec (apply concat histories))
        n      (count ops)
        ids    (volatile! {"null" -1})  ; :inspect leaders -> ids (lincheck.h: nil = "null" = -1)
        lid    (fn [x] (let [nm (leader-name x)]
                         (or (@ids nm) (let [i (dec (count @ids))] (vswap! ids assoc nm i) i))))
        off    (long-array (reductions + 0 (map count histories)))
        index  (long-array n) process (int-array n) types (byte-array n) fs (byte-array n)
        v0     (long-array n) v1 (long-array n) vflags (byte-array n)]
    (dotimes [i n]
      (let [op (nth ops i) v (:value op)]
        (aset index i (long (:index op i)))
        (aset process i (int (:process op)))
        (aset types i (byte (type-code (:type op))))
        (aset fs i (byte (f-code (:f op))))
        (cond (nil? v)    (aset vflags i (byte 0))
              (= :inspect (:f op))  ; [leader term ...] (leader.clj:14-17, :69)
                          (do (aset vflags i (byte 2))
                              (aset v0 i (long (lid (nth v 0))))
                              (aset v1 i (long (nth v 1))))
              (vector? v) (do (aset vflags i (byte 2))
                              (aset v0 i (long (v 0)))
                              (aset v1 i (long (v 1))))
              :else       (do (aset vflags i (byte 1)) (aset v0 i (long v))))))
    {:off off :index index :process process :types types :fs fs :v0 v0 :v1 v1 :vflags vflags}))

(defn- client-ops [history] (filterv #(integer? (:process %)) history))

(defn- failure-configs
  "lc_failure_configs (ABI 2) for history i of the lc_check this thread just made: up to k
  pre-failure configs as {:model {:value v} :linearized [inv-index ...] :last-op ok-index
  :pending [inv-index ...]} (:pending = every pending op; the config's own are those not in
  :linearized), plus the frontier's newest last op, or nil when the frontier could not be
  dumped (the verdict stands)."
  [i k]
  (let [state (long-array k) nils (byte-array k) lin (long-array (* 64 k)) n-lin (int-array k)
        last-op (long-array k) n-out (int-array 1) pending (long-array 64) n-pending (int-array 1)
        newest (long-array 1) err (byte-array 512)
        rc (.invokeInt (lib-fn "lc_failure_configs")
                       (object-array [(int i) (int k) state nils lin n-lin last-op n-out pending
                                      n-pending newest err (int 512)]))]
    (when (zero? rc)
      (let [pend (vec (take (aget n-pending 0) pending))]
        {:newest-last-op (aget newest 0)
         :configs (vec (for [c (range (aget n-out 0))]
                         {:model      {:value (when (zero? (aget nils c)) (aget state c))}
                          :linearized (vec (for [x (range (aget n-lin c))] (aget lin (+ (* 64 c) x))))
                          :last-op    (aget last-op c)
                          :pending    pend}))}))))

(defn- folded-ops
  "invocation :index -> the op as the model steps it (an :ok completion's :value folded into
  its invocation, as knossos.history/complete does)."
  [ops]
  (loop [ops ops, open {}, out {}]
    (if-let [o (first ops)]
      (let [p (:process o)]
        (if (= :invoke (:type o))
          (recur (rest ops) (assoc open p (:index o)) (assoc out (:index o) o))
          (let [i (open p)]
            (recur (rest ops) (dissoc open p)
                   (if (and i (= :ok (:type o))) (assoc-in out [i :value] (:value o)) out)))))
      out)))

(defn- leader-config-models
  "LeaderModel configs: the device reports each config's contested (term, leader) pairs only,
  so its model is rebuilt as the search defines it: (LeaderModel. {}) stepped through every op
  that returned :ok before the failing completion, then the pending ops the config linearized
  (a consistent map holds one leader per term, so the order does not matter)."
  [m configs ops fail-idx]
  (let [folded   (folded-ops ops)
        returned (loop [os ops, open {}, out []]
                   (let [o (first os)]
                     (if (or (nil? o) (= fail-idx (:index o)))
                       out
                       (let [p (:process o)]
                         (if (= :invoke (:type o))
                           (recur (rest os) (assoc open p (:index o)) out)
                           (recur (rest os) (dissoc open p)
                                  (if (and (open p) (= :ok (:type o))) (conj out (open p)) out)))))))]
    (vec (for [c configs]
           (assoc c :model (reduce (fn [mm i] (model/step mm (folded i)))
                                   m (concat returned (sort (:linearized c)))))))))

(defn- final-paths
  ":final-paths: from each pre-failure config, pending ops linearized one after another (each
  step consistent), ending with the failing op's inconsistent step; breadth-first, <= k."
  [m configs fail-inv ops k]
  (let [folded  (folded-ops ops)
        fop     (folded fail-inv)
        pending (sort (:pending (first configs)))]
    (when fop
      (loop [queue (for [c configs]
                     [(if (satisfies? model/Model (:model c))  ; LeaderModel: the rebuilt record
                        (:model c)
                        (assoc m :value (get-in c [:model :value])))
                      (set (:linearized c))
                      [{:op nil :model (:model c)}]])
             paths []]
        (if (or (empty? queue) (>= (count paths) k))
          (vec (take k paths))
          (let [done (for [[mm _ path] queue
                           :let [r (model/step mm fop)]
                           :when (model/inconsistent? r)]
                       (conj path {:op fop :model r}))
                nxt  (for [[mm lin path] queue
                           i pending
                           :when (and (not (lin i)) (not= i fail-inv) (folded i))
                           :let [r (model/step mm (folded i))]
                           :when (not (model/inconsistent? r))]
                       [r (conj lin i) (conj path {:op (folded i) :model r})])]
            (recur nxt (into paths done))))))))

(defn check-histories
  "One lc_check call for many histories; returns a vector of Knossos-keyed maps."
  [model-kind init histories opts]
  (let [{:keys [off index process types fs v0 v1 vflags]} (encode histories)
        k        (count histories)
        valid    (byte-array k) fail (long-array k) finv (long-array k) prev (long-array k)
        explored (long-array k) errs (int-array k) err (byte-array 512)
        rc       (.invokeInt (lib-fn "lc_check")
                             (object-array [(int model-kind) (long init) (int k) off index process
                                            types fs v0 v1 vflags (int (:gpus opts 0))
                                            (long (:max-configs opts 0)) (int 0) valid fail finv
                                            prev explored errs err (int 512)]))]
    (when-not (zero? rc)
      (throw (ex-info (c-string err) {:rc rc})))
    (vec (for [i (range k)]
           (let [ops (nth histories i)
                 ;; :index -> op, built once per history (was an O(n) filter per lookup)
                 by-index (persistent! (reduce (fn [m op] (assoc! m (:index op) op)) (transient {}) ops))
                 at  (fn [idx] (get by-index idx))
                 v   (aget valid i)]
             (cond-> {:valid?   (case v 1 true 0 false :unknown)
                      :analyzer :linear
                      :explored (aget explored i)}
               (= 2 v)    (assoc :error (get err-text (aget errs i) "undecided"))
               (zero? v)  (assoc :op          (at (aget fail i))
                                 :previous-ok (at (aget prev i))
                                 ;; without a report: every config the previous RETURN's JIT
                                 ;; closure emitted has the previous :ok op last
                                 :last-op     (at (aget prev i)))
               (and (zero? v) (:configs opts true))
               ((fn [r]
                  (if-let [{:keys [configs newest-last-op]}
                           ;; (some->: no report (LC_E_CONFIGS) keeps the :previous-ok fallback)
                           (some-> (failure-configs i 10)
                                   (cond-> (= 3 model-kind)
                                     (update :configs #(leader-config-models (:model opts) % ops
                                                                             (aget fail i)))))]
                    (cond-> (assoc r
                                   :last-op (at newest-last-op)
                                   ;; Knossos :configs: {:model :last-op :pending}, :pending =
                                   ;; the calls this config has not linearized
                                   :configs (vec (for [c configs
                                                       :let [lin (set (:linearized c))]]
                                                   {:model   (:model c)
                                                    :last-op (at (:last-op c))
                                                    :pending (vec (for [p (sort (:pending c))
                                                                        :when (not (lin p))]
                                                                    (at p)))})))
                      (seq configs) (assoc :final-paths
                                           (final-paths (:model opts) configs (aget finv i) ops 10)))
                    r)))))))))

(defn check-partitioned
  "ONE history with its frontier partitioned over n-ranks ranks of this process (lc_part_check:
  rank r on device r mod visible devices, candidates moved by peer copies over xGMI): for a
  history whose frontier outgrows one GPU (SURVEY §8(e) axis 2, e.g. the counter path's whole
  history at counter.clj:133-137 when registered as a cas-register). Same map as
  check-histories gives, without the failure report."
  [history n-ranks]
  (let [ops   (client-ops history)
        {:keys [off index process types fs v0 v1 vflags]} (encode [ops])
        valid (byte-array 1) fail (long-array 1) finv (long-array 1) prev (long-array 1)
        explored (long-array 1) errs (int-array 1) err (byte-array 512)
        rc    (.invokeInt (lib-fn "lc_part_check")
                          (object-array [(int 1) (long 0) (long (count ops)) index process types fs
                                         v0 v1 vflags (int n-ranks) (int 0) valid fail finv prev
                                         explored errs err (int 512)]))]
    (when-not (zero? rc)
      (throw (ex-info (c-string err) {:rc rc})))
    (let [at (fn [idx] (first (filter #(= idx (:index %)) ops)))
          v  (aget valid 0)]
      (cond-> {:valid? (case v 1 true 0 false :unknown) :analyzer :linear :explored (aget explored 0)}
        (= 2 v)   (assoc :error (get err-text (aget errs 0) "undecided"))
        (zero? v) (assoc :op (at (aget fail 0)) :previous-ok (at (aget prev 0))
                         :last-op (at (aget prev 0)))))))

(defn- model-kind
  "[model_kind init] for the models the GPU implements, else nil (-> Knossos)."
  [m]
  (cond (and (instance? CASRegister m) (nil? (:value m))) [1 0]  ; (model/cas-register)
        (= "CounterModel" (.getSimpleName (class m)))       [2 (long (:value m))]
        (and (= "LeaderModel" (.getSimpleName (class m)))     ; (LeaderModel. {}), leader.clj:84
             (empty? (:state m)))                            [3 0]
        :else nil))


(defn linearizable
  "Same options as checker/linearizable. Models the GPU does not implement (a cas-register with
  a non-nil initial value, a LeaderModel that does not start empty) fall back to Knossos."
  [{:keys [model] :as opts}]
  (if-let [[kind init] (model-kind model)]
    (reify checker/Checker
      (check [_ test history copts]
        (first (check-histories kind init [(client-ops history)] opts))))
    (checker/linearizable opts)))

(defn independent-checker
  "Batched drop-in for register.clj:106-111,
    (independent/checker (checker/compose {:timeline (timeline/html)
                                           :linear (checker/linearizable opts)}))
  Splits the history by key (jepsen.independent/history-keys, subhistory), sends EVERY key
  down in one lc_check, runs the other per-key checkers (e.g. {:timeline (timeline/html)})
  as compose would, and returns {:valid? :results {k {:linear .. :timeline ..}} :failures}.
  Falls back to the per-key independent/checker when the model is not a GPU model."
  ([opts] (independent-checker opts {}))
  ([{:keys [model] :as opts} others]
   (if-let [[kind init] (model-kind model)]
     (reify checker/Checker
       (check [_ test history copts]
         (let [ks      (vec (independent/history-keys history))
               subs    (mapv #(client-ops (independent/subhistory % history)) ks)
               linears (if (seq ks) (check-histories kind init subs opts) [])
               results (into {}
                             (map (fn [k sub lin]
                                    (let [kopts (assoc copts :subdirectory ["independent" k]
                                                             :history-key k)
                                          r     (into {:linear lin}
                                                      (for [[n c] others]
                                                        [n (checker/check-safe c test sub kopts)]))]
                                      [k (assoc r :valid? (checker/merge-valid (map :valid? (vals r))))]))
                                  ks subs linears))]
           {:valid?   (checker/merge-valid (map :valid? (vals results)))
            :results  results
            ;; jepsen.independent: keys whose :valid? is falsey (:unknown is truthy)
            :failures (vec (for [[k r] results :when (false? (:valid? r))] k))})))
     (independent/checker (checker/compose (assoc others :linear (checker/linearizable opts)))))))
